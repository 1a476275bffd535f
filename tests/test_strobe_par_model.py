"""Model check of the replay's parallel append (merlin_group.cuh
GroupStrobe::append32_par, GRP_PAR_APPEND): the masks its lanes XOR into the
sponge, one dword each, equal the byte-serial STROBE framing + absorb of
append_message(label, 32 bytes) (frame_fast + absorb32; merlin 3.0.0's
Transcript::append_message over STROBE-128, transcript_protocol.rs:26-47) for
every sponge position where both end before the rate and every label length
the replay uses.  CPU only: the lane formulas restated in Python."""
import random

R = 166  # STROBE-128 rate (merlin_lane.cuh LANE_STROBE_R)


def _alignbit(hi, lo, s):
    return ((((hi << 32) | lo) >> (s & 31)) & 0xFFFFFFFF)


def _serial(st, pos, pos_begin, label, w):
    st = bytearray(st)
    frame = bytes([pos_begin & 0xFF, 18]) + label + bytes([32, 0, 0, 0, (pos + 1) & 0xFF, 2])
    msg = b"".join(x.to_bytes(4, "little") for x in w)
    for i, b in enumerate(frame + msg):
        st[pos + i] ^= b
    return bytes(st)


def _parallel(st, pos, pos_begin, label, w):
    st = bytearray(st)
    ln = len(label)
    fl = 8 + ln
    fd = [0, 0, 0]

    def putb(i, v):
        fd[i >> 2] |= (v & 0xFF) << (8 * (i & 3))

    putb(0, pos_begin)
    putb(1, 18)
    for i in range(ln):
        putb(2 + i, label[i])
    putb(2 + ln, 32)
    putb(6 + ln, pos + 1)
    putb(7 + ln, 2)
    o = pos & 3
    for g in range(16):  # the group's lanes
        fcur = fd[g] if g < 3 else 0
        fprev = fd[g - 1] if 1 <= g <= 3 else 0
        m = _alignbit(fcur, fprev, 32 - 8 * o) if o else fcur
        v = 4 * g - o - fl
        qd, r = v >> 2, v & 3
        lo = w[qd] if 0 <= qd < 8 else 0
        hi = w[qd + 1] if 0 <= qd + 1 < 8 else 0
        m |= _alignbit(hi, lo, 8 * r)
        if g < 12:
            d = (pos >> 2) + g
            st[4 * d:4 * d + 4] = (int.from_bytes(st[4 * d:4 * d + 4], "little") ^ m).to_bytes(4, "little")
        else:
            assert m == 0
    return bytes(st)


def test_parallel_append_equals_serial():
    rng = random.Random(7)
    for ln in (1, 2, 3):
        for pos in range(0, R - (8 + ln + 32)):
            label = bytes(rng.choice(b"ABCDEFGHIJKLMNOPQRSTUVWXYZ_") for _ in range(ln))
            st = bytes(rng.randrange(256) for _ in range(256))
            w = [rng.getrandbits(32) for _ in range(8)]
            pb = rng.randrange(256)
            assert _parallel(st, pos, pb, label, w) == _serial(st, pos, pb, label, w), (ln, pos)
