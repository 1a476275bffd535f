"""Host-side Merlin transcript of libbpperm (C++ STROBE-128 / Keccak-f[1600],
no GPU needed) against the Merlin 3.0.0 known-answer test and the oracle's
restatement on randomized message sequences, including multi-block
challenges (the SHAKE/STROBE squeeze across permutation boundaries)."""
import random

import pytest

from oracle import merlin, ristretto as r255


@pytest.fixture(scope="module")
def bp():
    import bpperm
    bpperm._lib.load()
    return bpperm


def test_merlin_kat(bp):
    t = bp.Transcript(b"test protocol")
    t.append_message(b"some label", b"some data")
    assert t.challenge_bytes(b"challenge", 32).hex() == \
        "d5a21972d0d5fe320c0d263fac7fffb8145aa640af6e9bca177c03c7efcf0615"


@pytest.mark.parametrize("seed", range(6))
def test_transcript_matches_oracle(bp, seed):
    rng = random.Random(seed)
    label = bytes(rng.randrange(256) for _ in range(rng.randrange(1, 40)))
    o = merlin.Transcript(label)
    t = bp.Transcript(label)
    for _ in range(rng.randrange(3, 12)):
        op = rng.randrange(4)
        lab = bytes(rng.randrange(97, 123) for _ in range(rng.randrange(1, 12)))
        if op == 0:
            msg = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 700)))
            o.append_message(lab, msg)
            t.append_message(lab, msg)
        elif op == 1:
            x = rng.randrange(2 ** 64)
            o.append_u64(lab, x)
            t.append_u64(lab, x)
        elif op == 2:
            n = rng.choice([1, 32, 64, 135, 136, 137, 300])
            assert t.challenge_bytes(lab, n) == o.challenge_bytes(lab, n)
        else:
            assert t.challenge_scalar(lab) == r255.scalar_bytes(o.challenge_scalar(lab))
