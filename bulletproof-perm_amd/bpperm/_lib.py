"""ctypes binding of libbpperm.so (the C ABI declared in include/bpperm.h).

The product path has no CPU fallback: if the HIP library is missing or no
GPU is visible, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

# BPP_LIB selects an alternative build (A/B kernel experiments, build.py --variant)
LIB_PATH = Path(os.environ["BPP_LIB"]) if os.environ.get("BPP_LIB") else \
    Path(__file__).resolve().parent / "libbpperm.so"

BPP_OK = 0
ERRORS = {
    1: "BPP_ERR_ARG",
    2: "BPP_ERR_LEN",
    3: "BPP_ERR_DECOMPRESS",
    4: "BPP_ERR_NONCANONICAL",
    5: "BPP_ERR_DEVICE",
    6: "BPP_ERR_VERIFY",
    7: "BPP_ERR_NOMEM",
    8: "BPP_ERR_CALLBACK",
}

vp = C.c_void_p
sz = C.c_size_t
u8p = C.c_char_p
i32 = C.c_int
u32 = C.c_uint32
u64 = C.c_uint64

# name -> (restype, argtypes); keep in sync with include/bpperm.h
SIGNATURES = {
    "bpp_ctx_create": (i32, [i32, C.POINTER(vp)]),
    "bpp_ctx_destroy": (None, [vp]),
    "bpp_ctx_last_error": (C.c_char_p, [vp]),
    "bpp_ctx_stream": (vp, [vp]),
    "bpp_ctx_profile": (i32, [vp, i32]),
    "bpp_ctx_profile_get": (i32, [vp, C.c_char_p, C.POINTER(C.c_double), C.POINTER(u64)]),
    "bpp_ctx_profile_reset": (None, [vp]),
    "bpp_ctx_work_get": (i32, [vp, C.c_char_p, C.POINTER(u64)]),
    "bpp_ctx_work_reset": (None, [vp]),
    "bpp_host_tuning": (i32, [u32]),
    "bpp_host_threads": (u32, []),
    "bpp_dev_alloc": (i32, [vp, sz, C.POINTER(vp)]),
    "bpp_dev_free": (i32, [vp, vp]),
    "bpp_memcpy_htod": (i32, [vp, vp, vp, sz]),
    "bpp_memcpy_dtoh": (i32, [vp, vp, vp, sz]),
    "bpp_synchronize": (i32, [vp]),
    "bpp_points_decompress": (i32, [vp, vp, sz, C.POINTER(vp), C.POINTER(sz)]),
    "bpp_points_from_uniform": (i32, [vp, vp, sz, C.POINTER(vp)]),
    "bpp_points_compress": (i32, [vp, vp, vp]),
    "bpp_points_len": (sz, [vp]),
    "bpp_points_destroy": (None, [vp]),
    "bpp_msm": (i32, [vp, vp, vp, sz, vp]),
    "bpp_msm_table": (i32, [vp, vp, vp, sz, vp]),
    "bpp_msm_table_dev": (i32, [vp, vp, vp, sz, vp]),
    "bpp_msm_windows": (i32, [sz, C.POINTER(u32), C.POINTER(u32)]),
    "bpp_msm_table_dev_partial": (i32, [vp, vp, vp, sz, u32, u32, vp]),
    "bpp_msm_submit": (i32, [vp, vp, vp, sz, u32, u32, C.POINTER(C.c_uint64)]),
    "bpp_msm_collect": (i32, [vp, C.c_uint64, vp, vp]),
    "bpp_msm_submit_host": (i32, [vp, vp, vp, sz, u32, u32, C.POINTER(C.c_uint64)]),
    "bpp_host_alloc": (i32, [vp, sz, C.POINTER(vp)]),
    "bpp_host_free": (i32, [vp, vp]),
    "bpp_partials_finish": (i32, [vp, sz, vp]),
    "bpp_points_double_compress": (i32, [vp, sz, vp]),
    "bpp_msm_batch": (i32, [vp, sz, vp, vp, vp, vp, vp]),
    "bpp_gens_create": (i32, [vp, sz, C.POINTER(vp)]),
    "bpp_gens_from_points": (i32, [vp, vp, vp, sz, vp, vp, C.POINTER(vp)]),
    "bpp_gens_len": (sz, [vp]),
    "bpp_gens_export": (i32, [vp, vp, vp]),
    "bpp_gens_destroy": (None, [vp]),
    "bpp_pedersen_commit_batch": (i32, [vp, vp, vp, vp, sz, vp]),
    "bpp_vec_commit": (i32, [vp, vp, vp, vp, vp, sz, vp]),
    "bpp_transcript_new": (vp, [vp, sz]),
    "bpp_transcript_clone": (vp, [vp]),
    "bpp_transcript_destroy": (None, [vp]),
    "bpp_transcript_append_message": (i32, [vp, vp, sz, vp, sz]),
    "bpp_transcript_append_u64": (i32, [vp, vp, sz, u64]),
    "bpp_transcript_challenge_bytes": (i32, [vp, vp, sz, vp, sz]),
    "bpp_transcript_challenge_scalar": (i32, [vp, vp, sz, vp]),
    "bpp_ipa_prove": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, sz, vp, vp, vp, vp]),
    "bpp_ipa_verify": (i32, [vp, vp, vp, sz, vp, vp, vp, vp, vp, vp, vp, vp]),
    "bpp_ipa_prove_cb": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, sz, vp, vp, vp, vp]),
    "bpp_ipa_verify_cb": (i32, [vp, vp, vp, sz, vp, vp, vp, vp, vp, vp, vp, vp]),
    "bpp_perm_proof_len": (sz, [u32]),
    "bpp_perm_prove": (i32, [vp, vp, u32, u64, vp, sz, vp, vp, vp]),
    "bpp_perm_prove_batch": (i32, [vp, vp, u32, sz, vp, vp, sz, vp, vp]),
    "bpp_perm_prove_batch_entropy": (i32, [vp, vp, u32, sz, vp, vp, sz, vp, vp]),
    "bpp_debug_secret_residue": (i32, [vp, vp]),
    "bpp_perm_verify": (i32, [vp, vp, u32, vp, sz, vp, sz, vp]),
    "bpp_perm_verify_batch": (i32, [vp, vp, u32, sz, vp, sz, vp, vp]),
    "bpp_perm_verify_begin": (i32, [u32, sz, vp, sz, vp, vp, vp, C.POINTER(vp)]),
    "bpp_perm_verify_begin_dev": (i32, [vp, u32, sz, vp, sz, vp, vp, vp, C.POINTER(vp)]),
    "bpp_perm_verify_terms": (i32, [vp, C.POINTER(sz)]),
    "bpp_verify_seed": (i32, [vp]),
    "bpp_scalar_invert": (i32, [vp, vp]),
    "bpp_scalar_powers": (i32, [vp, sz, vp]),
    "bpp_perm_verify_scalars": (i32, [vp, vp, sz, vp, vp]),
    "bpp_perm_verify_partial": (i32, [vp, vp, vp, vp, sz, u32, u32, vp]),
    "bpp_perm_verify_slice_bytes": (sz, [vp]),
    "bpp_perm_verify_slice_scalars_at": (i32, [vp, vp, vp, sz, vp]),
    "bpp_perm_verify_begin_dev_async": (i32, [vp, u32, sz, vp, sz, vp, vp, vp]),
    "bpp_perm_verify_slice_point_bytes": (sz, [vp]),
    "bpp_perm_verify_slice_points": (i32, [vp, vp, vp]),
    "bpp_perm_verify_partial_sharded": (i32, [vp, vp, vp, sz, vp, sz, vp, sz, vp, sz, u32, u32, vp]),
    "bpp_perm_verify_end": (None, [vp]),
    "bpp_partials_is_identity": (i32, [vp, sz]),
}

_lib = None


def load(path: os.PathLike | None = None):
    """Load libbpperm.so (raises if it has not been built)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path else LIB_PATH
    if not p.exists():
        raise RuntimeError(f"libbpperm.so not built at {p}; run python bulletproof-perm_amd/build.py")
    lib = C.CDLL(str(p))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


class BppError(RuntimeError):
    def __init__(self, code: int, where: str, detail: str = ""):
        self.code = code
        self.name = ERRORS.get(code, f"code {code}")
        super().__init__(f"{where}: {self.name}{(': ' + detail) if detail else ''}")


def check(rc: int, where: str, ctx=None):
    if rc != BPP_OK:
        detail = ""
        if ctx is not None:
            try:
                detail = (load().bpp_ctx_last_error(ctx) or b"").decode()
            except Exception:  # pragma: no cover
                pass
        raise BppError(rc, where, detail)
