"""The inner-product argument over the CALLER's transcript (bpp_ipa_prove_cb /
bpp_ipa_verify_cb, include/bpperm.h): the library calls back into a
transcript it does not own at exactly bulletproofs 4.0.0's points
(innerproduct_domain_sep, append_point L / R, challenge_scalar u;
transcript_protocol.rs:26-67), so the Rust crate can keep its
merlin::Transcript (north_star; hook fields circuit_lib.rs:62-63).

The caller-owned transcript here is the ORACLE's merlin (oracle/merlin.py, an
independent pure-Python STROBE-128) behind ctypes hooks: L, R, a, b must
equal the config-2 golden (tests/golden/protocol.json) and the oracle's
ipa_create, the call sequence must be bulletproofs' exactly, and the
transcript must carry on after the IPA in the state the oracle's own IPA
leaves."""
import sys
from pathlib import Path

import pytest

from oracle import bulletproofs as bp, merlin, ristretto as r255
from oracle.merlin import Rng

pytestmark = pytest.mark.gpu
GOLD_DIR = Path(__file__).parent / "golden"
sb = r255.scalar_bytes


class Recording:
    """A caller-owned transcript (the oracle's) that logs every hook call."""

    def __init__(self, label: bytes, fail_at: int | None = None):
        self.t = merlin.Transcript(label)
        self.log = []
        self.fail_at = fail_at

    def _tick(self):
        if self.fail_at is not None and len(self.log) == self.fail_at:
            raise RuntimeError("hook failure injected")

    def append_message(self, label: bytes, msg: bytes):
        self._tick()
        self.log.append(("append", label, msg))
        self.t.append_message(label, msg)

    def challenge_bytes(self, label: bytes, n: int) -> bytes:
        self._tick()
        self.log.append(("challenge", label, n))
        return self.t.challenge_bytes(label, n)


def expected_log(n, L, R):
    log = [("append", b"dom-sep", b"ipp v1"), ("append", b"n", n.to_bytes(8, "little"))]
    for Lj, Rj in zip(L, R):
        log += [("append", b"L", Lj), ("append", b"R", Rj), ("challenge", b"u", 64)]
    return log


@pytest.fixture(scope="module")
def gens16(ctx):
    import bpperm
    g = bpperm.Gens(ctx, 16)
    yield g
    g.close()


@pytest.mark.parametrize("n", [1, 2, 16])
def test_ipa_prove_cb_oracle_transcript(ctx, gens16, n):
    import bpperm
    rng = Rng(700 + n)
    oG, oH = merlin.bulletproof_gens(16)
    G, H = oG[:n], oH[:n]
    Q = rng.point()
    a = [rng.scalar() for _ in range(n)]
    b = [rng.scalar() for _ in range(n)]
    gf = [rng.scalar() for _ in range(n)]
    hf = [rng.scalar() for _ in range(n)]
    ref_tr = merlin.Transcript(b"hooks")
    want = bp.ipa_create(ref_tr, Q, gf, hf, G, H, a, b)
    tr = Recording(b"hooks")
    L, R, ga, gb = gens16.ipa_prove(tr, r255.encode(Q), [sb(x) for x in gf], [sb(x) for x in hf],
                                    [sb(x) for x in a], [sb(x) for x in b])
    assert L == want.L and R == want.R and ga == sb(want.a) and gb == sb(want.b)
    assert tr.log == expected_log(n, L, R)
    # the caller's transcript carries on where the oracle's IPA left its own
    assert tr.t.challenge_bytes(b"after", 32) == ref_tr.challenge_bytes(b"after", 32)

    P = bp.msm([x * f for x, f in zip(a, gf)] + [x * f for x, f in zip(b, hf)] + [bp.inner(a, b)], G + H + [Q])
    args = (n, [sb(x) for x in gf], [sb(x) for x in hf], r255.encode(P), r255.encode(Q), L, R, ga, gb)
    tv = Recording(b"hooks")
    assert gens16.ipa_verify(tv, *args)
    assert tv.log == expected_log(n, L, R)
    # interoperable with the library's own Merlin either way
    assert gens16.ipa_verify(bpperm.Transcript(b"hooks"), *args)
    bad = list(args)
    bad[7] = sb((want.a + 1) % r255.L)
    assert not gens16.ipa_verify(Recording(b"hooks"), *bad)
    if n > 1:
        assert not gens16.ipa_verify(Recording(b"other"), *args)
        # validate_and_append_point: an identity L_0 is refused before it is appended
        bad = list(args)
        bad[5] = [bytes(32)] + L[1:]
        tz = Recording(b"hooks")
        assert not gens16.ipa_verify(tz, *bad)
        assert tz.log == expected_log(n, L, R)[:2]


def test_ipa_cb_hook_failure_aborts(ctx, gens16):
    """A hook that fails aborts the call (BPP_ERR_CALLBACK at the ABI; the
    Python binding re-raises the hook's own exception); the context stays
    usable."""
    import ctypes as C

    import bpperm
    rng = Rng(77)
    n = 8
    Q = r255.encode(rng.point())
    a = [sb(rng.scalar()) for _ in range(n)]
    b = [sb(rng.scalar()) for _ in range(n)]
    for at in (0, 1, 3, 4, 7):
        with pytest.raises(RuntimeError, match="hook failure injected"):
            gens16.ipa_prove(Recording(b"f", fail_at=at), Q, None, None, a, b)
    # at the ABI: the hook's nonzero return is BPP_ERR_CALLBACK
    h = bpperm.transcript_hooks(Recording(b"f", fail_at=2))
    lo, ro = C.create_string_buffer(96), C.create_string_buffer(96)
    ao, bo = C.create_string_buffer(32), C.create_string_buffer(32)
    ab, bb = b"".join(a), b"".join(b)
    rc = ctx.lib.bpp_ipa_prove_cb(ctx.h, gens16.h, C.byref(h.s), C.c_char_p(Q), None, None, C.c_char_p(ab),
                                  C.c_char_p(bb), n, lo, ro, ao, bo)
    assert rc == 8 and isinstance(h.error, RuntimeError)
    # no hooks, or a NULL hook, is an argument error, not a crash
    rc = ctx.lib.bpp_ipa_prove_cb(ctx.h, gens16.h, None, C.c_char_p(Q), None, None, C.c_char_p(ab),
                                  C.c_char_p(bb), n, lo, ro, ao, bo)
    assert rc == 1
    h2 = bpperm.transcript_hooks(Recording(b"f"))
    h2.s.challenge_bytes = type(h2.fc)()  # NULL function pointer
    rc = ctx.lib.bpp_ipa_prove_cb(ctx.h, gens16.h, C.byref(h2.s), C.c_char_p(Q), None, None, C.c_char_p(ab),
                                  C.c_char_p(bb), n, lo, ro, ao, bo)
    assert rc == 1
    # still usable
    tr = Recording(b"f")
    L, R, ga, gb = gens16.ipa_prove(tr, Q, None, None, a, b)
    assert len(L) == 3 and tr.log == expected_log(n, L, R)


def test_ipa_prove_noncanonical_input_then_exact(ctx, gens16):
    """A non-canonical a, b or factor fails bpp_ipa_prove with
    BPP_ERR_NONCANONICAL after Q's table build was queued (the call drains it
    before releasing the Q slot); the next call, with another Q, equals the
    oracle's proof."""
    import bpperm
    rng = Rng(91)
    n = 16
    oG, oH = merlin.bulletproof_gens(16)
    a = [rng.scalar() for _ in range(n)]
    b = [rng.scalar() for _ in range(n)]
    hf = [rng.scalar() for _ in range(n)]
    bad = (r255.L + 3).to_bytes(32, "little")
    for which in range(3):
        aa = [sb(x) for x in a]
        bb = [sb(x) for x in b]
        hh = [sb(x) for x in hf]
        (aa, bb, hh)[which][5] = bad
        with pytest.raises(bpperm.BppError) as ei:
            gens16.ipa_prove(bpperm.Transcript(b"nc"), r255.encode(rng.point()), None, hh, aa, bb)
        assert ei.value.name == "BPP_ERR_NONCANONICAL"
    Q = rng.point()
    want = bp.ipa_create(merlin.Transcript(b"nc"), Q, [1] * n, hf, oG[:n], oH[:n], a, b)
    tr = bpperm.Transcript(b"nc")
    L, R, ga, gb = gens16.ipa_prove(tr, r255.encode(Q), None, [sb(x) for x in hf], [sb(x) for x in a],
                                    [sb(x) for x in b])
    tr.close()
    assert L == want.L and R == want.R and ga == sb(want.a) and gb == sb(want.b)


def test_config2_ipa_through_caller_transcript(ctx):
    """Config 2 (n = 2^10 commitment + IPA) with the caller's transcript
    behind the hooks from the first message on: A appended and y drawn by the
    caller, the IPA through bpp_ipa_prove_cb -- L, R, a, b equal the golden;
    bpp_ipa_verify_cb accepts and refuses a tampered a."""
    import json

    import bpperm
    sys.path.insert(0, str(GOLD_DIR))
    from make_golden import config2_inputs
    c2 = json.loads((GOLD_DIR / "protocol.json").read_text())["config2"]
    n = c2["n"]
    aL, aR, alpha, Qraw, G, H, _ = config2_inputs(n, c2["seed"])
    g = bpperm.Gens(ctx, n)
    try:
        A = g.vec_commit(sb(alpha), [sb(x) for x in aL], [sb(x) for x in aR])
        assert A.hex() == c2["A"]
        tr = Recording(b"config2")
        tr.t.append_point(b"A", A)
        y = tr.t.challenge_scalar(b"y")
        yinv = bp.powers(r255.scalar_inv(y), n)
        Qp = r255.from_uniform_bytes(Qraw)
        Q = r255.encode(Qp)
        hf = [sb(x) for x in yinv]
        L, R, a, b = g.ipa_prove(tr, Q, None, hf, [sb(x) for x in aL], [sb(x) for x in aR])
        assert [x.hex() for x in L] == c2["L"] and [x.hex() for x in R] == c2["R"]
        assert a.hex() == c2["a"] and b.hex() == c2["b"]
        assert tr.log == expected_log(n, L, R)
        # P = <aL, G> + <aR o y^-i, H> + <aL, aR> Q, one GPU MSM over the exported generators
        Ge, He, _, _ = g.export()
        psc = aL + [(x * h) % r255.L for x, h in zip(aR, yinv)] + [bp.inner(aL, aR)]
        P = ctx.msm(b"".join(sb(x) for x in psc), b"".join(Ge + He + [Q]))
        for tamper in (0, 1):
            tv = Recording(b"config2")
            tv.t.append_point(b"A", A)
            tv.t.challenge_scalar(b"y")
            av = bytes([a[0] ^ tamper]) + a[1:]
            assert g.ipa_verify(tv, n, None, hf, P, Q, L, R, av, b) == (tamper == 0)
    finally:
        g.close()


def test_config2_flag_wait_fallback_subprocess():
    """The rounds' completion-flag wait with a 1-us spin budget
    (BPP_IPA_SPIN_US=1): every round falls back to the event wait after the
    flag spin, and config 2 still equals its golden (bench_config2's check),
    in a child process so the environment is read fresh."""
    import os
    import subprocess
    root = Path(__file__).resolve().parent.parent
    env = dict(os.environ, BPP_IPA_SPIN_US="1")
    r = subprocess.run([sys.executable, str(root / "tools" / "config2_once.py"), "3"], capture_output=True, text=True,
                       timeout=180, env=env, cwd=str(root))
    assert r.returncode == 0, (r.stdout + r.stderr)[-2000:]
    assert r.stdout.strip().split()[-1] == "True", r.stdout[-500:]
