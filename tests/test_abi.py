"""The C-ABI library builds, loads and exports every symbol include/*.h
declares (no compute calls: this runs without a GPU)."""
import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def declared_symbols():
    syms = set()
    for h in (ROOT / "include").glob("*.h"):
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        for m in re.finditer(r"^\s*(?:[A-Za-z_][\w\s\*]*?)\b(bpp_\w+)\s*\(", text, flags=re.M):
            syms.add(m.group(1))
    return sorted(syms)


def test_header_declares_api():
    syms = declared_symbols()
    assert "bpp_msm" in syms and "bpp_ctx_create" in syms
    assert len(syms) >= 20


def test_library_exports_every_declared_symbol():
    from bpperm import _lib
    lib = ctypes.CDLL(str(_lib.LIB_PATH))
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_covers_header():
    from bpperm import _lib
    missing = [s for s in declared_symbols() if s not in _lib.SIGNATURES]
    assert not missing, missing


def test_no_cpu_fallback_without_library(tmp_path):
    from bpperm import _lib
    with pytest.raises(RuntimeError):
        _lib.load(tmp_path / "missing.so")


def test_argument_checks_without_device():
    """Entry points reject bad arguments before any device call: a null
    context, k outside [2, 2^20], a null job (BPP_ERR_ARG = 1)."""
    from bpperm import _lib
    lib = ctypes.CDLL(str(_lib.LIB_PATH))
    ARG = 1
    lib.bpp_perm_proof_len.restype = ctypes.c_size_t
    assert lib.bpp_perm_proof_len(ctypes.c_uint32(1)) == 0
    assert lib.bpp_perm_proof_len(ctypes.c_uint32(0x7FFFFFFF)) == 0  # (2k would wrap)
    assert lib.bpp_perm_proof_len(ctypes.c_uint32((1 << 20) + 1)) == 0
    assert lib.bpp_perm_proof_len(ctypes.c_uint32(52)) > 0
    job = ctypes.c_void_p()
    buf = ctypes.create_string_buffer(64)
    for k in (0, 1, (1 << 20) + 1, 0xFFFFFFFF):
        assert lib.bpp_perm_verify_begin(ctypes.c_uint32(k), ctypes.c_size_t(0), None, ctypes.c_size_t(0), None,
                                         None, None, ctypes.byref(job)) == ARG
    for k in (2, 52):  # a null context is refused before the device is touched
        assert lib.bpp_perm_verify(None, None, ctypes.c_uint32(k), None, ctypes.c_size_t(0), buf,
                                   ctypes.c_size_t(64), buf) == ARG
        assert lib.bpp_perm_verify_batch(None, None, ctypes.c_uint32(k), ctypes.c_size_t(1), None,
                                         ctypes.c_size_t(0), buf, buf) == ARG
        assert lib.bpp_perm_prove(None, None, ctypes.c_uint32(k), ctypes.c_uint64(1), None, ctypes.c_size_t(0),
                                  buf, buf, None) == ARG
    assert lib.bpp_perm_verify_terms(None, ctypes.byref(ctypes.c_size_t())) == ARG
    # the empty host job: zero proofs, replayed nowhere
    assert lib.bpp_perm_verify_begin(ctypes.c_uint32(52), ctypes.c_size_t(0), None, ctypes.c_size_t(0), None, None,
                                     None, ctypes.byref(job)) == 0
    terms = ctypes.c_size_t()
    assert lib.bpp_perm_verify_terms(job, ctypes.byref(terms)) == 0
    assert terms.value == 2 * 128 + 2
    lib.bpp_perm_verify_end(job)


def test_host_exceptions_do_not_cross_the_abi():
    """A host allocation sized by the caller's arguments that cannot be met
    comes back as BPP_ERR_NOMEM (7) instead of a C++ exception unwinding
    into the caller (bpp_guard, csrc/ctx.h)."""
    from bpperm import _lib
    lib = ctypes.CDLL(str(_lib.LIB_PATH))
    job = ctypes.c_void_p()
    buf = ctypes.create_string_buffer(64)
    rc = lib.bpp_perm_verify_begin(ctypes.c_uint32(52), ctypes.c_size_t(1 << 40), None, ctypes.c_size_t(0), buf,
                                   buf, None, ctypes.byref(job))
    assert rc == 7 and not job.value


def test_scalar_helpers_match_python():
    """bpp_scalar_invert / bpp_scalar_powers (the caller-side algebra of the
    IPA's H_factors, circuit_lib.rs:274 and util.rs:138-157 exp_iter) equal
    Python big-integer arithmetic; zero and non-canonical inputs are refused
    (host-only entry points: no GPU)."""
    import hashlib

    import bpperm
    from bpperm._lib import BppError
    L = 2**252 + 27742317777372353535851937790883648493
    for i in range(8):
        x = int.from_bytes(hashlib.sha256(b"scalar-%d" % i).digest(), "little") % L
        xb = x.to_bytes(32, "little")
        assert int.from_bytes(bpperm.scalar_invert(xb), "little") == pow(x, -1, L)
        pw = bpperm.scalar_powers(xb, 37)
        assert [int.from_bytes(pw[32 * j: 32 * j + 32], "little") for j in range(37)] == [pow(x, j, L) for j in range(37)]
    assert bpperm.scalar_powers((5).to_bytes(32, "little"), 0) == b""
    with pytest.raises(BppError):
        bpperm.scalar_invert(bytes(32))
    with pytest.raises(BppError):
        bpperm.scalar_powers(L.to_bytes(32, "little"), 3)


def test_partials_refuse_unwritten_partial():
    """a 128-B partial whose Z is zero (an all-zero buffer a failed
    rank never wrote) absorbed the sum and encoded as the identity, so one
    such partial made bpp_partials_is_identity accept any batch.  It is now
    refused: bpp_partials_finish -> BPP_ERR_ARG, bpp_partials_is_identity ->
    BPP_ERR_VERIFY.  Host-only entry points (no GPU)."""
    from bpperm import _lib
    from oracle import ristretto as r255
    lib = ctypes.CDLL(str(_lib.LIB_PATH))
    P = r255.ed_mul(12345, r255.BASEPOINT)
    Pn = r255.ed_neg(P)
    raw = r255.raw_point_bytes
    zero = bytes(128)
    out = ctypes.create_string_buffer(32)

    def is_id(*parts):
        b = b"".join(parts)
        return lib.bpp_partials_is_identity(ctypes.c_char_p(b), ctypes.c_size_t(len(parts)))

    assert is_id(raw(r255.IDENTITY)) == 0
    assert is_id(raw(P), raw(Pn)) == 0
    assert is_id(raw(P)) == 6
    assert is_id(zero) == 6
    assert is_id(raw(P), raw(Pn), zero) == 6
    assert is_id(zero, raw(P), raw(Pn)) == 6
    assert lib.bpp_partials_finish(ctypes.c_char_p(zero), ctypes.c_size_t(1), out) == 1
    assert lib.bpp_partials_finish(ctypes.c_char_p(raw(P)), ctypes.c_size_t(1), out) == 0
    assert out.raw == r255.encode(P)


def test_integration_lists_every_export():
    """INTEGRATION.md §5 lists every export the header
    declares (and no retired one)."""
    sec = (ROOT / "INTEGRATION.md").read_text().split("## 5.")[1]
    syms = declared_symbols()
    assert [s for s in syms if f"`{s}`" not in sec] == []
    for gone in ("bpp_perm_verify_begin_dev_slice", "bpp_perm_verify_partial_gathered"):
        assert gone not in syms


def test_host_tuning_hw_queues_flag():
    """bpp_host_tuning(BPP_TUNE_HW_QUEUES) sets GPU_MAX_HW_QUEUES=8 for the
    process unless the caller set it (a production prover's queue count,
    VERDICT r5 weak 8); unknown flags are refused.  In a child process: the
    variable is process-wide."""
    import subprocess
    import sys
    code = ("import ctypes, os, sys; sys.path.insert(0, %r); from bpperm import _lib; "
            "lib = ctypes.CDLL(str(_lib.LIB_PATH)); "
            "assert lib.bpp_host_tuning(ctypes.c_uint32(4)) == 1; "
            "assert lib.bpp_host_tuning(ctypes.c_uint32(2)) == 0; "
            "libc = ctypes.CDLL(None); libc.getenv.restype = ctypes.c_char_p; "
            "print(libc.getenv(b'GPU_MAX_HW_QUEUES').decode())") % str(ROOT / "bulletproof-perm_amd")
    import os
    env = {k: v for k, v in os.environ.items() if k != "GPU_MAX_HW_QUEUES"}
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=60)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "8"
    env["GPU_MAX_HW_QUEUES"] = "4"
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=60)
    assert r.stdout.strip() == "4"  # the caller's own setting wins
