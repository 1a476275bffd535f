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

__all__ = ["Context", "PointTable", "BppError", "vartime_multiscalar_mul", "default_context"]


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
    """A point table resident in HBM (affine-Niels, 96 B / point)."""

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

    def msm_batch(self, offsets: Sequence[int], scalars, point_idx: Sequence[int], table: PointTable) -> list[bytes]:
        count = len(offsets) - 1
        s = _join(scalars, 32, "scalars")
        off = (C.c_uint64 * len(offsets))(*offsets)
        idx = (C.c_uint32 * max(1, len(point_idx)))(*point_idx)
        out = C.create_string_buffer(32 * max(count, 1))
        check(self.lib.bpp_msm_batch(self.h, count, off, _buf(s), idx, table.handle, out), "bpp_msm_batch", self.h)
        return [out.raw[32 * i: 32 * i + 32] for i in range(count)]


def msm_windows(n: int) -> tuple[int, int]:
    lib = _lib.load()
    c = C.c_uint32()
    w = C.c_uint32()
    lib.bpp_msm_windows(n, C.byref(c), C.byref(w))
    return c.value, w.value


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
