"""Keccak-f[1600] / STROBE-128 / Merlin transcript spec oracle — TEST ONLY.

Restates merlin 3.0.0 (not vendored; bp-perm/Cargo.lock) as used by the
reference's `TranscriptProtocol` (`bp-perm/src/transcript_protocol.rs:26-67`):

  arithmetic_domain_sep(n)   transcript_protocol.rs:27-30
  append_scalar              transcript_protocol.rs:32-34
  append_point               transcript_protocol.rs:45-47
  validate_and_append_point  transcript_protocol.rs:48-60
  challenge_scalar           transcript_protocol.rs:62-67  (64 B -> mod l)

Pinned by the Merlin "simple transcript" KAT (tests/test_oracle_kat.py);
Keccak-f is cross-checked against hashlib.sha3_256.
"""
from __future__ import annotations

import hashlib
import struct

from . import ristretto as r255

_RC = [
    0x0000000000000001, 0x0000000000008082, 0x800000000000808A, 0x8000000080008000,
    0x000000000000808B, 0x0000000080000001, 0x8000000080008081, 0x8000000000008009,
    0x000000000000008A, 0x0000000000000088, 0x0000000080008009, 0x000000008000000A,
    0x000000008000808B, 0x800000000000008B, 0x8000000000008089, 0x8000000000008003,
    0x8000000000008002, 0x8000000000000080, 0x000000000000800A, 0x800000008000000A,
    0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008,
]
_ROT = [
    [0, 36, 3, 41, 18],
    [1, 44, 10, 45, 2],
    [62, 6, 43, 15, 61],
    [28, 55, 25, 21, 56],
    [27, 20, 39, 8, 14],
]
_M64 = (1 << 64) - 1


def _rol(x, n):
    n %= 64
    return ((x << n) | (x >> (64 - n))) & _M64 if n else x


def keccak_f1600(state: bytearray) -> None:
    """In-place Keccak-f[1600] on a 200-byte state (lanes little-endian)."""
    A = [[0] * 5 for _ in range(5)]
    for x in range(5):
        for y in range(5):
            A[x][y] = int.from_bytes(state[8 * (x + 5 * y): 8 * (x + 5 * y) + 8], "little")
    for rnd in range(24):
        C = [A[x][0] ^ A[x][1] ^ A[x][2] ^ A[x][3] ^ A[x][4] for x in range(5)]
        Dd = [C[(x - 1) % 5] ^ _rol(C[(x + 1) % 5], 1) for x in range(5)]
        for x in range(5):
            for y in range(5):
                A[x][y] ^= Dd[x]
        B = [[0] * 5 for _ in range(5)]
        for x in range(5):
            for y in range(5):
                B[y][(2 * x + 3 * y) % 5] = _rol(A[x][y], _ROT[x][y])
        for x in range(5):
            for y in range(5):
                A[x][y] = B[x][y] ^ ((~B[(x + 1) % 5][y]) & B[(x + 2) % 5][y])
        A[0][0] ^= _RC[rnd]
    for x in range(5):
        for y in range(5):
            state[8 * (x + 5 * y): 8 * (x + 5 * y) + 8] = A[x][y].to_bytes(8, "little")


def sha3_256_via_f(msg: bytes) -> bytes:
    """SHA3-256 built on keccak_f1600, used only to self-check the permutation."""
    rate = 136
    st = bytearray(200)
    m = bytearray(msg) + b"\x06" + b"\x00" * ((rate - (len(msg) + 1) % rate) % rate)
    m[-1] |= 0x80
    for off in range(0, len(m), rate):
        for i in range(rate):
            st[i] ^= m[off + i]
        keccak_f1600(st)
    return bytes(st[:32])


# ---------------------------------------------------------------- STROBE-128
STROBE_R = 166
FLAG_I, FLAG_A, FLAG_C, FLAG_T, FLAG_M, FLAG_K = 1, 2, 4, 8, 16, 32


class Strobe128:
    def __init__(self, protocol_label: bytes):
        st = bytearray(200)
        st[0:6] = bytes([1, STROBE_R + 2, 1, 0, 1, 96])
        st[6:18] = b"STROBEv1.0.2"
        keccak_f1600(st)
        self.state = st
        self.pos = 0
        self.pos_begin = 0
        self.cur_flags = 0
        self.meta_ad(protocol_label, False)

    def clone(self) -> "Strobe128":
        c = Strobe128.__new__(Strobe128)
        c.state = bytearray(self.state)
        c.pos, c.pos_begin, c.cur_flags = self.pos, self.pos_begin, self.cur_flags
        return c

    def _run_f(self):
        self.state[self.pos] ^= self.pos_begin
        self.state[self.pos + 1] ^= 0x04
        self.state[STROBE_R + 1] ^= 0x80
        keccak_f1600(self.state)
        self.pos = 0
        self.pos_begin = 0

    def _absorb(self, data: bytes):
        for b in data:
            self.state[self.pos] ^= b
            self.pos += 1
            if self.pos == STROBE_R:
                self._run_f()

    def _squeeze(self, n: int) -> bytes:
        out = bytearray(n)
        for i in range(n):
            out[i] = self.state[self.pos]
            self.state[self.pos] = 0
            self.pos += 1
            if self.pos == STROBE_R:
                self._run_f()
        return bytes(out)

    def _begin_op(self, flags: int, more: bool):
        if more:
            assert self.cur_flags == flags
            return
        assert flags & FLAG_T == 0
        old_begin = self.pos_begin
        self.pos_begin = self.pos + 1
        self.cur_flags = flags
        self._absorb(bytes([old_begin, flags]))
        force_f = (flags & (FLAG_C | FLAG_K)) != 0
        if force_f and self.pos != 0:
            self._run_f()

    def meta_ad(self, data: bytes, more: bool):
        self._begin_op(FLAG_M | FLAG_A, more)
        self._absorb(data)

    def ad(self, data: bytes, more: bool):
        self._begin_op(FLAG_A, more)
        self._absorb(data)

    def prf(self, n: int, more: bool) -> bytes:
        self._begin_op(FLAG_I | FLAG_A | FLAG_C, more)
        return self._squeeze(n)


# ---------------------------------------------------------------- Merlin
class Transcript:
    """merlin 3.0.0 `Transcript` plus the reference's TranscriptProtocol."""

    def __init__(self, label: bytes):
        self.strobe = Strobe128(b"Merlin v1.0")
        self.append_message(b"dom-sep", label)

    def clone(self) -> "Transcript":
        t = Transcript.__new__(Transcript)
        t.strobe = self.strobe.clone()
        return t

    def append_message(self, label: bytes, message: bytes):
        self.strobe.meta_ad(label, False)
        self.strobe.meta_ad(struct.pack("<I", len(message)), True)
        self.strobe.ad(message, False)

    def append_u64(self, label: bytes, x: int):
        self.append_message(label, struct.pack("<Q", x))

    def challenge_bytes(self, label: bytes, n: int) -> bytes:
        self.strobe.meta_ad(label, False)
        self.strobe.meta_ad(struct.pack("<I", n), True)
        return self.strobe.prf(n, False)

    # --- TranscriptProtocol (transcript_protocol.rs) ---
    def arithmetic_domain_sep(self, n: int):  # :27-30
        self.append_message(b"dom-sep", b"acp v1")
        self.append_u64(b"n", n)

    def innerproduct_domain_sep(self, n: int):  # bulletproofs 4.0.0
        self.append_message(b"dom-sep", b"ipp v1")
        self.append_u64(b"n", n)

    def append_scalar(self, label: bytes, s: int):  # :32-34
        self.append_message(label, r255.scalar_bytes(s))

    def append_point(self, label: bytes, compressed: bytes):  # :45-47
        self.append_message(label, compressed)

    def validate_and_append_point(self, label: bytes, compressed: bytes):  # :48-60
        if compressed == bytes(32):
            raise ValueError("VerificationError: identity point")
        self.append_message(label, compressed)

    def challenge_scalar(self, label: bytes) -> int:  # :62-67
        return r255.scalar_from_wide(self.challenge_bytes(label, 64))


# ---------------------------------------------------------------- generators
def pedersen_gens_default():
    """bulletproofs `PedersenGens::default()`: B = basepoint,
    B_blinding = RistrettoPoint::hash_from_bytes::<Sha3_512>(B.compress())."""
    B = r255.BASEPOINT
    h = hashlib.sha3_512(r255.encode(B)).digest()
    return B, r255.from_uniform_bytes(h)


def generators_chain(label: bytes, count: int, skip: int = 0):
    """bulletproofs `GeneratorsChain`: SHAKE256("GeneratorsChain" || label),
    64 bytes per point -> from_uniform_bytes.  (parity unpinned: recalled spec)"""
    xof = hashlib.shake_256(b"GeneratorsChain" + label).digest(64 * (skip + count))
    return [r255.from_uniform_bytes(xof[64 * (skip + i): 64 * (skip + i + 1)]) for i in range(count)]


def bulletproof_gens(n: int, party: int = 0):
    """`BulletproofGens::new(n, 1)` G_vec[party], H_vec[party]."""
    lab = struct.pack("<I", party)
    return generators_chain(b"G" + lab, n), generators_chain(b"H" + lab, n)


# ---------------------------------------------------------------- test RNG
class Rng:
    """Deterministic byte stream shared by the oracle and the product so that
    'random' blindings are reproducible: SHAKE256("bpperm-rng" || seed_le64).
    Stands in for the reference's `rand::thread_rng()` (circuit_lib.rs:175)."""

    def __init__(self, seed, domain: bytes = b"bpperm-rng"):
        # an int is the u64 test seed (8 bytes LE); bytes are taken as is
        # (the 32-byte entropy seeds of bpp_perm_prove_batch_entropy)
        sb = bytes(seed) if isinstance(seed, (bytes, bytearray)) else struct.pack("<Q", seed)
        self._xof = hashlib.shake_256(domain + sb)
        self._pos = 0
        self._buf = b""

    def bytes(self, n: int) -> bytes:
        need = self._pos + n
        if need > len(self._buf):
            self._buf = self._xof.digest(max(need, 2 * len(self._buf), 4096))
        out = self._buf[self._pos: need]
        self._pos = need
        return out

    def scalar(self) -> int:  # Scalar::random
        return r255.scalar_from_wide(self.bytes(64))

    def point(self):  # RistrettoPoint::random
        return r255.from_uniform_bytes(self.bytes(64))


def indexed_scalar(seed, j: int, domain: bytes = b"bpperm-prove-sc") -> int:
    """Draw j of a proof's blinding scalars: from_wide of the first 64 bytes of
    SHAKE256(domain || seed || le32(j)) (seed bytes as in Rng).  Every draw is
    its own one-block sponge, so the GPU makes each in its own thread
    (poly.hip k_draws) where one sequential stream would serialize them."""
    sb = bytes(seed) if isinstance(seed, (bytes, bytearray)) else struct.pack("<Q", seed)
    return r255.scalar_from_wide(hashlib.shake_256(domain + sb + struct.pack("<I", j)).digest(64))
