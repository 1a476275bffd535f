"""Pin the CPU oracle before trusting it.

The reference's own tests pin no numeric result, so parity is
anchored on published known-answer vectors for the third-party primitives the
reference calls (curve25519-dalek-ng 4.1.1, merlin 3.0.0, bulletproofs 4.0.0)
and on an independent in-container implementation (OpenSSL Ed25519)."""
import hashlib
import shutil
import subprocess

import pytest

from oracle import merlin, ristretto as r255

RFC9496_MULTIPLES = [
    "0000000000000000000000000000000000000000000000000000000000000000",
    "e2f2ae0a6abc4e71a884a961c500515f58e30b6aa582dd8db6a65945e08d2d76",
    "6a493210f7499cd17fecb510ae0cea23a110e8d5b901f8acadd3095c73a3b919",
    "94741f5d5d52755ece4f23f044ee27d5d1ea1e2bd196b462166b16152a9d0259",
    "da80862773358b466ffadfe0b3293ab3d9fd53c5ea6c955358f568322daf6a57",
    "e882b131016b52c1d3337080187cf768423efccbb517bb495ab812c4160ff44e",
    "f64746d3c92b13050ed8d80236a7f0007c3b3f962f5ba793d19a601ebb1df403",
    "44f53520926ec81fbd5a387845beb7df85a96a24ece18738bdcfa6a7822a176d",
    "903293d8f2287ebe10e2374dc1a53e0bc887e592699f02d077d5263cdd55601c",
    "02622ace8f7303a31cafc63f8fc48fdc16e1c8c8d234b2f0d6685282a9076031",
    "20706fd788b2720a1ed2a5dad4952b01f413bcf0e7564de8cdc816689e2db95f",
    "bce83f8ba5dd2fa572864c24ba1810f9522bc6004afe95877ac73241cafdab42",
    "e4549ee16b9aa03099ca208c67adafcafa4c3f3e4e5303de6026e3ca8ff84460",
    "aa52e000df2e16f55fb1032fc33bc42742dad6bd5a8fc0be0167436c5948501f",
    "46376b80f409b29dc2b5f6f0c52591990896e5716f41477cd30085ab7f10301e",
    "e0c418f7c8d9c4cdd7395b93ea124f3ad99021bb681dfc3302a9d99a2e53e64e",
]

# RFC 9496 §A.3 hash-to-group vector #1
H2G_IN = ("5d1be09e3d0c82fc538112490e35701979d99e06ca3e2b5b54bffe8b4dc772c1"
          "4d98b696a1bbfb5ca32c436cc61c16563790306c79eaca7705668b47dffe5bb6")
H2G_OUT = "3066f82a1a747d45120d1740f14358531a8f04bbffe6a819f86dfe50f44a0a46"

# RFC 9496 §A.2 bad encodings (a selection: non-canonical, negative, non-square)
BAD_ENCODINGS = [
    "00ffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff",
    "ffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
    "f3ffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
    "edffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
    "0100000000000000000000000000000000000000000000000000000000000000",
    "01ffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
    "26948d35ca62e643e26a83177332e6b6afeb9d08e4268b650f1f5bbd8d81d371",
    "4eac077a713c57b4f4397629a4145982c661f48044dd3f96427d40b147d9742f",
]


@pytest.mark.parametrize("k", range(16))
def test_rfc9496_basepoint_multiples(k):
    assert r255.encode(r255.ed_mul(k, r255.BASEPOINT)).hex() == RFC9496_MULTIPLES[k]


@pytest.mark.parametrize("k", range(16))
def test_rfc9496_decode_roundtrip(k):
    enc = bytes.fromhex(RFC9496_MULTIPLES[k])
    assert r255.encode(r255.decode(enc)) == enc


@pytest.mark.parametrize("h", BAD_ENCODINGS)
def test_rfc9496_bad_encodings_rejected(h):
    with pytest.raises(r255.DecodeError):
        r255.decode(bytes.fromhex(h))


def test_rfc9496_hash_to_group():
    assert r255.encode(r255.from_uniform_bytes(bytes.fromhex(H2G_IN))).hex() == H2G_OUT


def test_pedersen_gens_default_b_blinding():
    _, Bb = merlin.pedersen_gens_default()
    assert r255.encode(Bb).hex() == "8c9240b456a9e6dc65c377a1048d745f94a08cdb7f44cbcd7b46f34048871134"


def test_keccak_matches_hashlib():
    for msg in [b"", b"abc", bytes(range(200)), b"x" * 1000]:
        assert merlin.sha3_256_via_f(msg) == hashlib.sha3_256(msg).digest()


def test_merlin_simple_transcript_kat():
    t = merlin.Transcript(b"test protocol")
    t.append_message(b"some label", b"some data")
    assert t.challenge_bytes(b"challenge", 32).hex() == \
        "d5a21972d0d5fe320c0d263fac7fffb8145aa640af6e9bca177c03c7efcf0615"


def test_scalar_wide_reduction():
    assert r255.scalar_from_wide(bytes(64)) == 0
    assert r255.scalar_from_wide(b"\xff" * 64) == (2**512 - 1) % r255.L


def _edwards_encode(p):
    x, y = r255.ed_affine(p)
    return (y | ((x & 1) << 255)).to_bytes(32, "little")


@pytest.mark.skipif(shutil.which("openssl") is None, reason="openssl not installed")
def test_openssl_ed25519_cross_check(tmp_path):
    """Independent implementation of the same curve: Ed25519 public key of
    seed 00..1f from OpenSSL == [clamp(SHA-512(seed))]B from the oracle."""
    seed = bytes(range(32))
    der = bytes.fromhex("302e020100300506032b657004220420") + seed
    (tmp_path / "k.der").write_bytes(der)
    out = subprocess.run(["openssl", "pkey", "-inform", "DER", "-in", str(tmp_path / "k.der"),
                          "-pubout", "-outform", "DER"], capture_output=True, check=True).stdout
    pub = out[-32:]
    h = bytearray(hashlib.sha512(seed).digest()[:32])
    h[0] &= 248
    h[31] &= 127
    h[31] |= 64
    a = int.from_bytes(h, "little")
    assert _edwards_encode(r255.ed_mul(a, r255.BASEPOINT)) == pub
    assert pub.hex() == "03a107bff3ce10be1d70dd18e74bc09967e4d6309ba50d5f1ddc8664125531b8"
