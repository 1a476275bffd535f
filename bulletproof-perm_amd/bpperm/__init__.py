"""bpperm — MI355X-native Bulletproof permutation hot path (Python host side).

Thin host mirror of the reference's operator surface over the C ABI in
include/bpperm.h (libbpperm.so, HIP for gfx950):

  vartime_multiscalar_mul(scalars, points)   dalek VartimeMultiscalarMul
                                             (bp-perm/src/circuit_lib.rs:187…568)
  Context.decompress / PointTable.compress   CompressedRistretto::decompress,
                                             RistrettoPoint::compress
  Context.from_uniform                       RistrettoPoint::from_uniform_bytes

Scalars are 32-byte little-endian canonical values mod l; points are 32-byte
compressed ristretto255, exactly dalek's `as_bytes()` forms.  There is no
CPU fallback: without the built library or a GPU every call raises.
"""
from __future__ import annotations

import ctypes as C
from typing import Iterable, Sequence

from . import _lib
from ._lib import BppError, check

MSM_INFLIGHT = 4  # BPP_MSM_INFLIGHT (include/bpperm.h)

__all__ = ["Context", "PointTable", "BppError", "vartime_multiscalar_mul", "default_context", "VerifyJob",
           "partials_is_identity"]


def _buf(b: bytes):
    return C.c_char_p(b) if b else None


def _join(items: Iterable[bytes], width: int, what: str) -> bytes:
    if isinstance(items, (bytes, bytearray, memoryview)):
        data = bytes(items)
    else:
        data = b"".join(bytes(x) for x in items)
    if len(data) % width:
        raise ValueError(f"{what}: length {len(data)} not a multiple of {width}")
    return data


class PointTable:
    """A point table resident in HBM (affine Niels, 10-limb field, 128-B rows)."""

    def __init__(self, ctx: "Context", handle: int):
        self._ctx = ctx
        self._h = C.c_void_p(handle)

    def __len__(self) -> int:
        return int(self._ctx.lib.bpp_points_len(self._h))

    @property
    def handle(self):
        return self._h

    def compress(self) -> list[bytes]:
        n = len(self)
        out = C.create_string_buffer(32 * n) if n else None
        check(self._ctx.lib.bpp_points_compress(self._ctx.h, self._h, out), "bpp_points_compress", self._ctx.h)
        raw = out.raw if n else b""
        return [raw[32 * i: 32 * i + 32] for i in range(n)]

    def close(self):
        if self._h:
            self._ctx.lib.bpp_points_destroy(self._h)
            self._h = C.c_void_p(0)

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class Context:
    """One GPU + one HIP stream (bpp_ctx)."""

    def __init__(self, device: int = 0):
        self.lib = _lib.load()
        h = C.c_void_p()
        rc = self.lib.bpp_ctx_create(device, C.byref(h))
        if rc != 0:
            raise BppError(rc, f"bpp_ctx_create(device={device})")
        self.h = h
        self.device = device

    def close(self):
        if self.h:
            self.lib.bpp_ctx_destroy(self.h)
            self.h = C.c_void_p(0)

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def stream(self) -> int:
        return int(self.lib.bpp_ctx_stream(self.h) or 0)

    def secret_residue(self) -> int:
        """Nonzero bytes left in what the last production prover batch zeroed
        (bpp_debug_secret_residue; a test hook)."""
        nz = C.c_uint64()
        check(self.lib.bpp_debug_secret_residue(self.h, C.byref(nz)), "bpp_debug_secret_residue", self.h)
        return nz.value

    # ---------------------------------------------------------- profiling
    def profile(self, enable: bool = True):
        check(self.lib.bpp_ctx_profile(self.h, 1 if enable else 0), "bpp_ctx_profile", self.h)

    def profile_get(self, stage: str):
        ms = C.c_double()
        n = C.c_uint64()
        check(self.lib.bpp_ctx_profile_get(self.h, stage.encode(), C.byref(ms), C.byref(n)),
              "bpp_ctx_profile_get", self.h)
        return ms.value, n.value

    def profile_reset(self):
        self.lib.bpp_ctx_profile_reset(self.h)

    WORK_COUNTERS = ("msm_terms", "madds", "padds", "msm_launches", "dt_terms", "dt_madds", "dt_launches",
                     "ipa_dt_terms", "ipa_dt_madds", "ipa_dt_launches")

    def work(self) -> dict:
        """Algorithmic work issued on this context since the last work_reset
        (bpp_ctx_work_get): MSM terms, mixed additions, point additions."""
        out = {}
        for name in self.WORK_COUNTERS:
            v = C.c_uint64()
            check(self.lib.bpp_ctx_work_get(self.h, name.encode(), C.byref(v)), "bpp_ctx_work_get", self.h)
            out[name] = v.value
        return out

    def work_reset(self):
        self.lib.bpp_ctx_work_reset(self.h)

    # ---------------------------------------------------------- device memory
    def dev_alloc(self, nbytes: int) -> int:
        p = C.c_void_p()
        check(self.lib.bpp_dev_alloc(self.h, nbytes, C.byref(p)), "bpp_dev_alloc", self.h)
        return p.value

    def dev_free(self, ptr: int):
        check(self.lib.bpp_dev_free(self.h, C.c_void_p(ptr)), "bpp_dev_free", self.h)

    def htod(self, dptr: int, data: bytes):
        check(self.lib.bpp_memcpy_htod(self.h, C.c_void_p(dptr), _buf(data), len(data)), "bpp_memcpy_htod", self.h)

    def dtoh(self, dptr: int, nbytes: int) -> bytes:
        out = C.create_string_buffer(nbytes)
        check(self.lib.bpp_memcpy_dtoh(self.h, out, C.c_void_p(dptr), nbytes), "bpp_memcpy_dtoh", self.h)
        return out.raw

    def synchronize(self):
        check(self.lib.bpp_synchronize(self.h), "bpp_synchronize", self.h)

    # ---------------------------------------------------------- points
    def decompress(self, encodings) -> PointTable:
        data = _join(encodings, 32, "encodings")
        h = C.c_void_p()
        bad = C.c_size_t()
        check(self.lib.bpp_points_decompress(self.h, _buf(data), len(data) // 32, C.byref(h), C.byref(bad)),
              "bpp_points_decompress", self.h)
        return PointTable(self, h.value)

    def from_uniform(self, bytes64) -> PointTable:
        data = _join(bytes64, 64, "uniform bytes")
        h = C.c_void_p()
        check(self.lib.bpp_points_from_uniform(self.h, _buf(data), len(data) // 64, C.byref(h)),
              "bpp_points_from_uniform", self.h)
        return PointTable(self, h.value)

    # ---------------------------------------------------------- MSM
    def msm(self, scalars, points) -> bytes:
        """vartime_multiscalar_mul over host scalars and compressed points."""
        s = _join(scalars, 32, "scalars")
        p = _join(points, 32, "points")
        if len(s) // 32 != len(p) // 32:
            raise BppError(2, "bpp_msm", "scalar/point count mismatch")
        out = C.create_string_buffer(32)
        check(self.lib.bpp_msm(self.h, _buf(s), _buf(p), len(s) // 32, out), "bpp_msm", self.h)
        return out.raw

    def msm_table(self, scalars, table: PointTable, n: int | None = None) -> bytes:
        s = _join(scalars, 32, "scalars")
        n = len(s) // 32 if n is None else n
        out = C.create_string_buffer(32)
        check(self.lib.bpp_msm_table(self.h, _buf(s), table.handle, n, out), "bpp_msm_table", self.h)
        return out.raw

    def msm_table_dev(self, d_scalars: int, table: PointTable, n: int) -> bytes:
        out = C.create_string_buffer(32)
        check(self.lib.bpp_msm_table_dev(self.h, C.c_void_p(d_scalars), table.handle, n, out),
              "bpp_msm_table_dev", self.h)
        return out.raw

    def msm_table_dev_partial(self, d_scalars: int, table: PointTable, n: int, w_begin: int, w_end: int) -> bytes:
        out = C.create_string_buffer(128)
        check(self.lib.bpp_msm_table_dev_partial(self.h, C.c_void_p(d_scalars), table.handle, n, w_begin, w_end, out),
              "bpp_msm_table_dev_partial", self.h)
        return out.raw

    # Asynchronous single MSMs (at most two in flight): submit returns a
    # ticket at once; collect waits for it and returns the compressed result
    # (or the raw 128-byte partial of windows [w_begin, w_end)).
    def msm_submit(self, d_scalars: int, table: PointTable, n: int, w_begin: int = 0, w_end: int = 0) -> int:
        t = C.c_uint64()
        check(self.lib.bpp_msm_submit(self.h, C.c_void_p(d_scalars), table.handle, n, w_begin, w_end, C.byref(t)),
              "bpp_msm_submit", self.h)
        return t.value

    def msm_submit_host(self, h_scalars, table: PointTable, n: int, w_begin: int = 0, w_end: int = 0) -> int:
        """As msm_submit with host scalars: a pinned buffer address from
        host_alloc (int; direct DMA on the MSM's stream) or bytes (staged)."""
        t = C.c_uint64()
        ptr = C.c_void_p(h_scalars) if isinstance(h_scalars, int) else _buf(h_scalars)
        check(self.lib.bpp_msm_submit_host(self.h, ptr, table.handle, n, w_begin, w_end, C.byref(t)),
              "bpp_msm_submit_host", self.h)
        return t.value

    def host_alloc(self, nbytes: int) -> int:
        """Pinned host memory (bpp_host_alloc); free with host_free."""
        p = C.c_void_p()
        check(self.lib.bpp_host_alloc(self.h, nbytes, C.byref(p)), "bpp_host_alloc", self.h)
        return p.value

    def host_free(self, ptr: int):
        check(self.lib.bpp_host_free(self.h, C.c_void_p(ptr)), "bpp_host_free", self.h)

    def msm_collect(self, ticket: int, partial: bool = False) -> bytes:
        out = C.create_string_buffer(128 if partial else 32)
        args = (None, out) if partial else (out, None)
        check(self.lib.bpp_msm_collect(self.h, ticket, *args), "bpp_msm_collect", self.h)
        return out.raw

    def msm_batch(self, offsets: Sequence[int], scalars, point_idx: Sequence[int], table: PointTable) -> list[bytes]:
        count = len(offsets) - 1
        s = _join(scalars, 32, "scalars")
        off = (C.c_uint64 * len(offsets))(*offsets)
        idx = (C.c_uint32 * max(1, len(point_idx)))(*point_idx)
        out = C.create_string_buffer(32 * max(count, 1))
        check(self.lib.bpp_msm_batch(self.h, count, off, _buf(s), idx, table.handle, out), "bpp_msm_batch", self.h)
        raw = out.raw  # .raw copies the whole buffer on every access
        return [raw[32 * i: 32 * i + 32] for i in range(count)]


def host_tuning(malloc: bool = True, hw_queues: bool = False):
    """Opt-in process-wide host tuning (bpp_host_tuning): BPP_TUNE_MALLOC
    fixes glibc's mmap threshold and disables heap trimming (the prover's
    per-batch host vectors stay in the arenas); BPP_TUNE_HW_QUEUES asks HIP
    for 8 hardware queues (GPU_MAX_HW_QUEUES=8 unless set; effective only
    before anything in the process initialises HIP)."""
    check(_lib.load().bpp_host_tuning((1 if malloc else 0) | (2 if hw_queues else 0)), "bpp_host_tuning")


def host_pool_threads() -> int:
    """Threads of the library's host pool (bpp_host_threads)."""
    return int(_lib.load().bpp_host_threads())


def msm_windows(n: int) -> tuple[int, int]:
    lib = _lib.load()
    c = C.c_uint32()
    w = C.c_uint32()
    lib.bpp_msm_windows(n, C.byref(c), C.byref(w))
    return c.value, w.value


def double_compress(raw_points: Sequence[bytes]) -> list[bytes]:
    """compress(2 P) for raw 128-byte extended points (host batch encoding)."""
    lib = _lib.load()
    data = b"".join(raw_points)
    out = C.create_string_buffer(32 * len(raw_points))
    check(lib.bpp_points_double_compress(_buf(data), len(raw_points), out), "bpp_points_double_compress")
    return [out.raw[32 * i:32 * i + 32] for i in range(len(raw_points))]


def partials_finish(partials: Sequence[bytes]) -> bytes:
    lib = _lib.load()
    data = b"".join(partials)
    out = C.create_string_buffer(32)
    check(lib.bpp_partials_finish(_buf(data), len(partials), out), "bpp_partials_finish")
    return out.raw


_default: Context | None = None


def default_context() -> Context:
    global _default
    if _default is None:
        _default = Context(0)
    return _default


def vartime_multiscalar_mul(scalars, points) -> bytes:
    """`RistrettoPoint::vartime_multiscalar_mul(scalars, points).compress()`."""
    return default_context().msm(scalars, points)


# ------------------------------------------------------------------ protocol
class Transcript:
    """merlin 3.0.0 `Transcript` on the host side of libbpperm (byte-exact;
    transcript_protocol.rs TranscriptProtocol helpers included)."""

    def __init__(self, label: bytes = b"", _handle=None):
        self.lib = _lib.load()
        self.h = C.c_void_p(_handle) if _handle else C.c_void_p(self.lib.bpp_transcript_new(_buf(label), len(label)))

    def clone(self) -> "Transcript":
        return Transcript(_handle=self.lib.bpp_transcript_clone(self.h))

    def close(self):
        if self.h:
            self.lib.bpp_transcript_destroy(self.h)
            self.h = C.c_void_p(0)

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def append_message(self, label: bytes, msg: bytes):
        check(self.lib.bpp_transcript_append_message(self.h, _buf(label), len(label), _buf(msg), len(msg)),
              "append_message")

    def append_u64(self, label: bytes, x: int):
        check(self.lib.bpp_transcript_append_u64(self.h, _buf(label), len(label), x), "append_u64")

    def challenge_bytes(self, label: bytes, n: int) -> bytes:
        out = C.create_string_buffer(n)
        check(self.lib.bpp_transcript_challenge_bytes(self.h, _buf(label), len(label), out, n), "challenge_bytes")
        return out.raw

    def challenge_scalar(self, label: bytes) -> bytes:
        out = C.create_string_buffer(32)
        check(self.lib.bpp_transcript_challenge_scalar(self.h, _buf(label), len(label), out), "challenge_scalar")
        return out.raw

    # TranscriptProtocol (transcript_protocol.rs)
    def arithmetic_domain_sep(self, n: int):
        self.append_message(b"dom-sep", b"acp v1")
        self.append_u64(b"n", n)

    def append_scalar(self, label: bytes, s: bytes):
        self.append_message(label, s)

    def append_point(self, label: bytes, p: bytes):
        self.append_message(label, p)


# bpp_transcript_hooks (include/bpperm.h): the caller's transcript behind C hooks
_APPEND_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_ubyte), C.c_size_t, C.POINTER(C.c_ubyte), C.c_size_t)
_CHALLENGE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_ubyte), C.c_size_t, C.POINTER(C.c_ubyte), C.c_size_t)


class _Hooks(C.Structure):
    _fields_ = [("user", C.c_void_p), ("append_message", _APPEND_FN), ("challenge_bytes", _CHALLENGE_FN)]


def transcript_hooks(tr):
    """bpp_transcript_hooks over any object with merlin's two primitives,
    `append_message(label, msg)` and `challenge_bytes(label, n) -> bytes`
    (the caller keeps its own transcript, bpp_ipa_prove_cb).  An exception in
    a hook is kept on the returned object (`.error`) and reported to the
    library as a failed hook (BPP_ERR_CALLBACK)."""

    class _H:
        error = None

    h = _H()

    def _append(_u, lab, ll, msg, ml):
        try:
            tr.append_message(C.string_at(lab, ll), C.string_at(msg, ml) if ml else b"")
            return 0
        except Exception as e:  # noqa: BLE001 (reported through BPP_ERR_CALLBACK)
            h.error = e
            return 1

    def _challenge(_u, lab, ll, out, n):
        try:
            b = tr.challenge_bytes(C.string_at(lab, ll), n)
            if len(b) != n:
                raise ValueError("challenge_bytes returned %d bytes, wanted %d" % (len(b), n))
            C.memmove(out, b, n)
            return 0
        except Exception as e:  # noqa: BLE001
            h.error = e
            return 1

    h.fa, h.fc = _APPEND_FN(_append), _CHALLENGE_FN(_challenge)  # (kept alive with h)
    h.s = _Hooks(None, h.fa, h.fc)
    return h


def _tr_args(tr, lib, plain: str):
    """(function, transcript argument, hooks holder) for a library Transcript
    (bpp_transcript*) or a caller-owned one (hooks)."""
    if isinstance(tr, Transcript):
        return getattr(lib, plain), tr.h, None
    h = transcript_hooks(tr)
    return getattr(lib, plain + "_cb"), C.byref(h.s), h


class Gens:
    """BulletproofGens(n, 1) + PedersenGens resident on the GPU (bpp_gens)."""

    def __init__(self, ctx: Context, n: int | None = None, points=None):
        self.ctx = ctx
        h = C.c_void_p()
        if points is None:
            check(ctx.lib.bpp_gens_create(ctx.h, n, C.byref(h)), "bpp_gens_create", ctx.h)
        else:
            G, H, B, Bb = points
            g = _join(G, 32, "G")
            hh = _join(H, 32, "H")
            check(ctx.lib.bpp_gens_from_points(ctx.h, _buf(g), _buf(hh), len(g) // 32, _buf(B), _buf(Bb),
                                               C.byref(h)), "bpp_gens_from_points", ctx.h)
        self.h = h

    def __len__(self):
        return int(self.ctx.lib.bpp_gens_len(self.h))

    def export(self):
        n = len(self)
        out = C.create_string_buffer(32 * (2 * n + 2))
        check(self.ctx.lib.bpp_gens_export(self.ctx.h, self.h, out), "bpp_gens_export", self.ctx.h)
        raw = out.raw
        pts = [raw[32 * i: 32 * i + 32] for i in range(2 * n + 2)]
        return pts[:n], pts[n: 2 * n], pts[2 * n], pts[2 * n + 1]

    def close(self):
        if self.h:
            self.ctx.lib.bpp_gens_destroy(self.h)
            self.h = C.c_void_p(0)

    def pedersen_commit(self, v, gamma) -> list[bytes]:
        """PedersenGens::commit over a batch (weights.rs:58-61)."""
        vb = _join(v, 32, "v")
        gb = _join(gamma, 32, "gamma")
        m = len(vb) // 32
        if len(gb) // 32 != m:
            raise BppError(2, "bpp_pedersen_commit_batch", "length mismatch")
        out = C.create_string_buffer(32 * max(m, 1))
        check(self.ctx.lib.bpp_pedersen_commit_batch(self.ctx.h, self.h, _buf(vb), _buf(gb), m, out),
              "bpp_pedersen_commit_batch", self.ctx.h)
        raw = out.raw
        return [raw[32 * i: 32 * i + 32] for i in range(m)]

    def vec_commit(self, blind: bytes, a, b=None) -> bytes:
        ab = _join(a, 32, "a")
        bb = _join(b, 32, "b") if b is not None else None
        out = C.create_string_buffer(32)
        check(self.ctx.lib.bpp_vec_commit(self.ctx.h, self.h, _buf(blind), _buf(ab), _buf(bb) if bb else None,
                                          len(ab) // 32, out), "bpp_vec_commit", self.ctx.h)
        return out.raw

    def ipa_prove(self, tr, Q: bytes, G_factors, H_factors, a, b):
        """InnerProductProof::create -> (L list, R list, a, b).  `tr`: a
        bpperm.Transcript, or the caller's own transcript object (merlin's
        append_message / challenge_bytes; bpp_ipa_prove_cb)."""
        ab, bb = _join(a, 32, "a"), _join(b, 32, "b")
        n = len(ab) // 32
        gf = _join(G_factors, 32, "G_factors") if G_factors is not None else None
        hf = _join(H_factors, 32, "H_factors") if H_factors is not None else None
        lg = max(n.bit_length() - 1, 0)
        Lo = C.create_string_buffer(32 * max(lg, 1))
        Ro = C.create_string_buffer(32 * max(lg, 1))
        ao, bo = C.create_string_buffer(32), C.create_string_buffer(32)
        fn, targ, hooks = _tr_args(tr, self.ctx.lib, "bpp_ipa_prove")
        rc = fn(self.ctx.h, self.h, targ, _buf(Q), _buf(gf) if gf else None, _buf(hf) if hf else None, _buf(ab),
                _buf(bb), n, Lo, Ro, ao, bo)
        if hooks is not None and hooks.error is not None:
            raise hooks.error
        check(rc, "bpp_ipa_prove", self.ctx.h)
        lraw, rraw = Lo.raw, Ro.raw
        return ([lraw[32 * i: 32 * i + 32] for i in range(lg)], [rraw[32 * i: 32 * i + 32] for i in range(lg)],
                ao.raw, bo.raw)

    def ipa_verify(self, tr, n: int, G_factors, H_factors, P: bytes, Q: bytes, L, R, a: bytes,
                   b: bytes) -> bool:
        gf = _join(G_factors, 32, "G_factors") if G_factors is not None else None
        hf = _join(H_factors, 32, "H_factors") if H_factors is not None else None
        fn, targ, hooks = _tr_args(tr, self.ctx.lib, "bpp_ipa_verify")
        rc = fn(self.ctx.h, self.h, targ, n, _buf(gf) if gf else None, _buf(hf) if hf else None, _buf(P), _buf(Q),
                _buf(b"".join(L)), _buf(b"".join(R)), _buf(a), _buf(b))
        if hooks is not None and hooks.error is not None:
            raise hooks.error
        if rc == 6:
            return False
        check(rc, "bpp_ipa_verify", self.ctx.h)
        return True


class PermProver:
    """Permutation proof over resident generators — the sound-mode restatement
    of ACProof::ArithmeticCircuitProof (circuit_lib.rs:139-585)."""

    def __init__(self, gens: Gens, k: int, label: bytes = b"bp-perm", ctx: "Context | None" = None):
        """ctx: the context (stream, workspaces) proofs run on; default the
        generators' own.  One generator set may serve several contexts, e.g.
        one per host thread with batches in flight."""
        self.gens = gens
        self.ctx = ctx or gens.ctx
        self.k = k
        self.label = label
        self.proof_len = int(self.ctx.lib.bpp_perm_proof_len(k))
        self.m = 2 * k + 1

    def prove(self, seed: int):
        """-> (proof bytes, [V_j], permutation)"""
        pf = C.create_string_buffer(self.proof_len)
        V = C.create_string_buffer(32 * self.m)
        perm = (C.c_uint32 * self.k)()
        check(self.ctx.lib.bpp_perm_prove(self.ctx.h, self.gens.h, self.k, seed, _buf(self.label), len(self.label),
                                          pf, V, perm), "bpp_perm_prove", self.ctx.h)
        vraw = V.raw
        return pf.raw, [vraw[32 * j: 32 * j + 32] for j in range(self.m)], list(perm)

    def prove_batch(self, seeds: Sequence[int], raw: bool = False):
        """-> ([proof bytes], [V bytes of one proof]), or with raw=True the
        two contiguous buffers (proofs, V) as the C ABI writes them (what
        verify_batch takes without a join)."""
        cnt = len(seeds)
        pf = C.create_string_buffer(self.proof_len * cnt)
        V = C.create_string_buffer(32 * self.m * cnt)
        sd = (C.c_uint64 * cnt)(*seeds)
        check(self.ctx.lib.bpp_perm_prove_batch(self.ctx.h, self.gens.h, self.k, cnt, sd, _buf(self.label),
                                                len(self.label), pf, V), "bpp_perm_prove_batch", self.ctx.h)
        praw, vraw = pf.raw, V.raw
        if raw:
            return praw, vraw
        return ([praw[i * self.proof_len:(i + 1) * self.proof_len] for i in range(cnt)],
                [vraw[i * 32 * self.m:(i + 1) * 32 * self.m] for i in range(cnt)])

    def prove_batch_entropy(self, count: int, seeds32: bytes | None = None, raw: bool = False):
        """Production proving: 32 bytes of entropy per proof (seeds32) or,
        when None, from the OS CSPRNG (bpp_perm_prove_batch_entropy); the
        batch's secrets are wiped before it returns.  raw=True: the two
        contiguous buffers (proofs, V), as prove_batch(..., raw=True)."""
        if seeds32 is not None and len(seeds32) != 32 * count:
            raise ValueError("seeds32 must hold 32 bytes per proof")
        pf = C.create_string_buffer(self.proof_len * count)
        V = C.create_string_buffer(32 * self.m * count)
        check(self.ctx.lib.bpp_perm_prove_batch_entropy(self.ctx.h, self.gens.h, self.k, count, _buf(seeds32 or b""),
                                                        _buf(self.label), len(self.label), pf, V),
              "bpp_perm_prove_batch_entropy", self.ctx.h)
        praw, vraw = pf.raw, V.raw
        if raw:
            return praw, vraw
        return ([praw[i * self.proof_len:(i + 1) * self.proof_len] for i in range(count)],
                [vraw[i * 32 * self.m:(i + 1) * 32 * self.m] for i in range(count)])

    def verify(self, proof: bytes, V) -> bool:
        vb = _join(V, 32, "V")
        rc = self.ctx.lib.bpp_perm_verify(self.ctx.h, self.gens.h, self.k, _buf(self.label), len(self.label),
                                          _buf(proof), len(proof), _buf(vb))
        if rc == 6:
            return False
        check(rc, "bpp_perm_verify", self.ctx.h)
        return True

    def verify_batch(self, proofs, Vs) -> bool:
        """proofs / Vs: sequences of per-proof bytes, or the two contiguous
        buffers (prove_batch(..., raw=True))."""
        if isinstance(proofs, (bytes, bytearray)):
            pb, vb = bytes(proofs), bytes(Vs)
            count = len(pb) // self.proof_len
            if len(pb) != count * self.proof_len or len(vb) != count * 32 * self.m:
                raise ValueError("contiguous proofs / V buffers of inconsistent length")
        else:
            pb, vb, count = b"".join(proofs), b"".join(Vs), len(proofs)
        rc = self.ctx.lib.bpp_perm_verify_batch(self.ctx.h, self.gens.h, self.k, count, _buf(self.label),
                                                len(self.label), _buf(pb), _buf(vb))
        if rc == 6:
            return False
        check(rc, "bpp_perm_verify_batch", self.ctx.h)
        return True

    def verify_batch_ptr(self, proofs_ptr: int, V_ptr: int, count: int) -> bool:
        """verify_batch over `count` proofs and their V already in host
        memory at two addresses -- e.g. pinned buffers from
        Context.host_alloc, which go up by DMA without the staging copy."""
        rc = self.ctx.lib.bpp_perm_verify_batch(self.ctx.h, self.gens.h, self.k, count, _buf(self.label),
                                                len(self.label), C.c_void_p(proofs_ptr), C.c_void_p(V_ptr))
        if rc == 6:
            return False
        check(rc, "bpp_perm_verify_batch", self.ctx.h)
        return True

    def verify_job(self, proofs: Sequence[bytes], Vs: Sequence[bytes], device: bool = True) -> "VerifyJob":
        """Replay phase of a batch verification that may be split over GPUs:
        on this prover's context (device=True, bpp_perm_verify_begin_dev) or
        on the host (bpp_perm_verify_begin)."""
        return VerifyJob(self.k, proofs, Vs, self.label, ctx=self.ctx if device else None)

    def verify_partial_sharded(self, job: "VerifyJob", first: int, d_blocks: int, stride: int, d_pblocks: int,
                               pstride: int, counts: Sequence[int], w_begin: int, w_end: int) -> bytes:
        """128-B raw partial of the whole batch's MSM over windows [w_begin,
        w_end), from every slice's scalar block (d_blocks + s * stride) and
        decompressed point block (d_pblocks + s * pstride) gathered in slice
        order; job = this rank's job over its own slice, batch proofs [first,
        first + job.count) (bpp_perm_verify_partial_sharded)."""
        part = C.create_string_buffer(128)
        cn = (C.c_size_t * max(len(counts), 1))(*counts)
        check(self.ctx.lib.bpp_perm_verify_partial_sharded(self.ctx.h, self.gens.h, job.h, first, d_blocks, stride,
                                                           d_pblocks, pstride, cn, len(counts), w_begin, w_end, part),
              "bpp_perm_verify_partial_sharded", self.ctx.h)
        return part.raw

    def verify_partial(self, job: "VerifyJob", seed: bytes, first: int, w_begin: int, w_end: int) -> bytes:
        """128-B raw partial of job's MSM over windows [w_begin, w_end) (see
        bpp_perm_verify_partial); seed = the batch's 32 verifier-random bytes
        (verify_seed(), the same on every rank), first = the batch index of
        the job's first proof.  None when a proof point does not decode
        (BPP_ERR_VERIFY)."""
        part = C.create_string_buffer(128)
        rc = self.ctx.lib.bpp_perm_verify_partial(self.ctx.h, self.gens.h, job.h, _seed(seed), first, w_begin, w_end,
                                                  part)
        if rc == 6:  # a proof point that does not decode: the batch cannot verify
            return None
        check(rc, "bpp_perm_verify_partial", self.ctx.h)
        return part.raw


class VerifyJob:
    """Parsed proofs with their transcripts replayed: on the host
    (bpp_perm_verify_begin, ctx=None; no GPU) or on the GPU of `ctx`
    (bpp_perm_verify_begin_dev: the job's records stay in that context's
    workspaces, valid until its next device job).  `r` holds each proof's
    weight challenge; proof p's batch weight mixes it with the batch's
    verifier seed (bpp_perm_verify_scalars)."""

    def __init__(self, k: int, proofs: Sequence[bytes], Vs: Sequence[bytes], label: bytes = b"bp-perm",
                 ctx: "Context | None" = None, wait: bool = True):
        """wait=False (a device job): bpp_perm_verify_begin_dev_async --
        returns before the replay ends, `r` is None and a rejected proof
        surfaces as False from slice_scalars / verify_partial."""
        self.lib = _lib.load()
        self.k = k
        self.count = len(proofs)
        self.device = ctx is not None
        self.ctx = ctx
        h = C.c_void_p()
        nr = self.count
        r = C.create_string_buffer(32 * nr + 1)
        pb, vb = _buf(b"".join(proofs)), _buf(b"".join(Vs))
        if ctx is None:
            rc = self.lib.bpp_perm_verify_begin(k, self.count, _buf(label), len(label), pb, vb, r, C.byref(h))
            name = "bpp_perm_verify_begin"
        elif not wait:
            self._keep = (pb, vb)  # (pinned inputs are read after the return; these are staged, but keep them)
            rc = self.lib.bpp_perm_verify_begin_dev_async(ctx.h, k, self.count, _buf(label), len(label), pb, vb,
                                                          C.byref(h))
            name = "bpp_perm_verify_begin_dev_async"
            nr = 0
        else:
            rc = self.lib.bpp_perm_verify_begin_dev(ctx.h, k, self.count, _buf(label), len(label), pb, vb, r,
                                                    C.byref(h))
            name = "bpp_perm_verify_begin_dev"
        if rc == 6:
            self.h = None
            self.r = None
            return
        check(rc, name, ctx.h if ctx is not None else None)
        self.h = h
        self.r = r.raw[:32 * nr] if nr else (None if not wait else b"")

    def slice_bytes(self) -> int:
        return int(self.lib.bpp_perm_verify_slice_bytes(self.h))

    def slice_scalars(self, seed: bytes, d_out: int, first: int = 0) -> bool:
        """The replayed slice's MSM scalars into device memory d_out
        (slice_bytes() bytes; bpp_perm_verify_slice_scalars_at), weighted from
        the batch's verifier seed; first = the batch index of the job's first
        proof.  False
        if an asynchronous begin's replay rejected a proof."""
        rc = self.lib.bpp_perm_verify_slice_scalars_at(self.ctx.h, self.h, _seed(seed), first, d_out)
        if rc == 6:
            return False
        check(rc, "bpp_perm_verify_slice_scalars_at", self.ctx.h)
        return True

    def point_bytes(self) -> int:
        """Bytes of the job's decompressed proof points (128 per point)."""
        return int(self.lib.bpp_perm_verify_slice_point_bytes(self.h))

    def slice_points(self, d_out: int) -> bool:
        """The job's decompressed proof points into device memory d_out
        (point_bytes() bytes; bpp_perm_verify_slice_points); False if a
        point did not decode."""
        rc = self.lib.bpp_perm_verify_slice_points(self.ctx.h, self.h, d_out)
        if rc == 6:
            return False
        check(rc, "bpp_perm_verify_slice_points", self.ctx.h)
        return True

    @property
    def ok(self) -> bool:
        """False if a proof was malformed (the batch cannot verify)."""
        return self.h is not None

    def terms(self) -> int:
        n = C.c_size_t()
        check(self.lib.bpp_perm_verify_terms(self.h, C.byref(n)), "bpp_perm_verify_terms")
        return n.value

    def windows(self) -> tuple[int, int]:
        return msm_windows(self.terms())

    def scalars(self, seed: bytes, first: int):
        """(scalars, proof-point encodings) of the job's MSM (host), its
        proofs being batch proofs [first, first + count) weighted from the
        batch's verifier seed: the first 2 n_p + 2 scalars go to G[0..n_p),
        H[0..n_p), B, B_blinding."""
        T = self.terms()
        n_p = 1
        while n_p < 2 * self.k:
            n_p <<= 1
        npts = T - (2 * n_p + 2)
        sc = C.create_string_buffer(32 * T)
        pts = C.create_string_buffer(32 * max(npts, 1))
        check(self.lib.bpp_perm_verify_scalars(self.h, _seed(seed), first, sc, pts), "bpp_perm_verify_scalars")
        sraw, praw = sc.raw, pts.raw
        return ([sraw[32 * i: 32 * i + 32] for i in range(T)], [praw[32 * i: 32 * i + 32] for i in range(npts)])

    def close(self):
        if self.h is not None:
            self.lib.bpp_perm_verify_end(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def scalar_invert(x: bytes) -> bytes:
    """Scalar::invert of a canonical 32-byte scalar (bpp_scalar_invert)."""
    out = C.create_string_buffer(32)
    check(_lib.load().bpp_scalar_invert(_buf(bytes(x)), out), "bpp_scalar_invert")
    return out.raw


def scalar_powers(x: bytes, n: int) -> bytes:
    """x^0 .. x^(n-1) as n x 32 bytes (bpp_scalar_powers; util.rs exp_iter)."""
    out = C.create_string_buffer(32 * max(n, 1))
    check(_lib.load().bpp_scalar_powers(_buf(bytes(x)), n, out), "bpp_scalar_powers")
    return out.raw[:32 * n]


def verify_seed() -> bytes:
    """32 bytes of verifier randomness for one batch (bpp_verify_seed: the OS
    CSPRNG).  Every job / rank of the batch must use the same bytes."""
    out = C.create_string_buffer(32)
    check(_lib.load().bpp_verify_seed(out), "bpp_verify_seed")
    return out.raw


def _seed(seed: bytes):
    if not isinstance(seed, (bytes, bytearray)) or len(seed) != 32:
        raise ValueError("a batch-verification seed is 32 bytes")
    return _buf(bytes(seed))


def partials_is_identity(partials: Sequence[bytes]) -> bool:
    """True iff the raw partial points add up to the identity."""
    raw = _join(partials, 128, "partial")
    rc = _lib.load().bpp_partials_is_identity(_buf(raw), len(partials))
    if rc == 6:
        return False
    check(rc, "bpp_partials_is_identity")
    return True

