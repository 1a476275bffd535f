"""The reference prover and verifier AS WRITTEN (compat mode) — TEST ONLY.

SURVEY.md §7 / §8(d) config 1 ask for the 52-card proof in both modes; the
product (and `bulletproofs.ac_prove`) is the SOUND form.  This module
restates the reference's one driver, `test_first` (bp-perm/src/lib.rs:
160-233), call for call, with every defect of SURVEY.md §2.2 that it
exercises kept:

  Q1  exp_iter yields Fibonacci exponents x, x, x^2, x^3, x^5, ...
      (util.rs:63-65,138-157) -> y_n, z_q
  Q2  create_weights returns Q x n matrices; create() asserts n x Q
      (circuit_lib.rs:157-173), so the only runnable form transposes them
      (weights.rs:203's commented-out transpose)
  Q3  create_a's chain join and a_O[n-1] = a_L^2 (weights.rs:63-113)
  Q4  T_i commits to t(i), the polynomial's VALUE at i, not its
      coefficient (circuit_lib.rs:362-412)
  Q5  the transcript gets T_3's bytes under label "T4" (circuit_lib.rs:391)
  Q6  tau_x adds x^2 <z_q, W_V gamma> five times (circuit_lib.rs:452-456)
  Q7  the final P == cand_P check is commented out (circuit_lib.rs:577-582)
  Q8  l, r go into the transcript as bytevec-encoded decimal strings
      (circuit_lib.rs:466-467, transcript_protocol.rs:36-43): bytevec
      0.2.0 is not in the container, so those bytes are UNPINNED; this
      restatement stops the transcript before that append and returns l, r
      as scalars (nothing after it draws a challenge)
  --  commit_variables blinds V with fresh randomness, unrelated to the
      gamma the prover later uses in tau_x (weights.rs:58-61 vs lib.rs:196)

and the verify of circuit_lib.rs:478-585 run on the prover's own state, as
the reference does, which fails at its second check ("IT ALREADY FAILS
HERE", circuit_lib.rs:541-543).

Randomness.  The reference draws everything from rand::thread_rng (lib.rs:
161-196, circuit_lib.rs:175-214, 360-404, weights.rs:37-61).  Here one
seeded stream `Rng(seed, b"bpperm-compat")` stands in, drawn in the
reference's order: B, B_blinding, the H_factors challenge, G[0..n),
H[0..n), the shuffle of [1..k] (Fisher-Yates; `shuffle::irs::Irs` is not
in the container), V's m blindings, gamma[0..m), alpha, beta, ro,
s_l[0..n), s_r[0..n), tau_1, tau_3 .. tau_6.  Points are
`RistrettoPoint::random` shaped (from_uniform_bytes of 64 stream bytes),
scalars `Scalar::random` shaped (from_bytes_mod_order_wide of 64).

Parity: the flow and quirks follow the cited lines; the numbers are
"parity unpinned" (the reference's randomness is not injectable and it
holds no fixtures).  tests/test_compat_prover.py runs the group operations
of this flow through the product's C ABI (MSMs, Pedersen commitments,
transcript) and compares them with this restatement.
"""
from __future__ import annotations

from dataclasses import dataclass, field

from . import ristretto as r255
from .bulletproofs import compat_create_a, compat_create_weights, compat_exp_iter, fisher_yates
from .merlin import Rng, Transcript

L = r255.L


def _transpose(m):  # weights.rs:115-129
    return [list(c) for c in zip(*m)]


def vm_mult(a, b):  # util.rs:22-37: out[i] = <a, b[i]>, len(a) == len(b[0])
    if len(a) != len(b[0]):
        raise ValueError("vm_mult: panics (dimension mismatch)")
    return [sum(x * y for x, y in zip(a, row)) % L for row in b]


def mv_mult(a, b):  # util.rs:39-53: out[i] = sum_j a[j][i] b[j], len(a) == len(b)
    if len(a) != len(b):
        raise ValueError("mv_mult: panics (dimension mismatch)")
    return [sum(a[j][i] * b[j] for j in range(len(b))) % L for i in range(len(a[0]))]


def hadamard(a, b):  # util.rs:6-20
    if len(a) != len(b):
        raise ValueError("hadamard_V: panics (dimension mismatch)")
    return [x * y % L for x, y in zip(a, b)]


def inner(a, b):  # util.rs:84-94
    if len(a) != len(b):
        raise ValueError("inner_product: panics (dimension mismatch)")
    return sum(x * y for x, y in zip(a, b)) % L


def scalar_exp(x, p):  # util.rs:74-81
    return pow(x, p, L)


def special_inner_product(l, r):  # poly.rs:39-58 (no <l1, r2>, <l2, r2> terms; r2 = 0 here)
    return [inner(l[1], r[0]),
            (inner(l[1], r[1]) + inner(l[2], r[0])) % L,
            (inner(l[2], r[1]) + inner(l[3], r[0])) % L,
            (inner(l[1], r[3]) + inner(l[3], r[1])) % L,
            inner(l[2], r[3]),
            inner(l[3], r[3])]


def poly6_eval(t, x):  # poly.rs:13-17: x (t1 + x (t2 + ... + x t6)), no constant term
    acc = 0
    for c in reversed(t):
        acc = (c + x * acc) % L
    return x * acc % L


def vecpoly3_eval(p, x):  # poly.rs:61-76
    return [(p[0][i] + x * (p[1][i] + x * (p[2][i] + x * p[3][i]))) % L for i in range(len(p[0]))]


@dataclass
class CompatRun:
    """Everything test_first computes up to the l / r append, plus the
    verify's intermediate group elements."""
    k: int
    n: int
    Q: int
    m: int
    B: tuple
    Bb: tuple
    G: list
    H: list
    v: list
    V_blind: list
    V: list                 # commit_variables (weights.rs:58-61)
    gamma: list
    aL: list
    aR: list
    aO: list
    WL: list                # transposed (n x Q), Q2
    WR: list
    WO: list
    WV: list                # m x Q
    c: list
    alpha: int
    beta: int
    ro: int
    s_l: list
    s_r: list
    A_I: tuple
    A_O: tuple
    S: tuple
    y: int
    z: int
    y_n: list
    y_n_inv: list
    z_q: list
    z_W_L: list
    z_W_R: list
    l_in: list
    sigma: int
    t_poly: list            # t1..t6 (Poly6)
    taus: list              # tau_1, tau_3, tau_4, tau_5, tau_6
    t_vals: list            # t(1), t(3), t(4), t(5), t(6) (Q4)
    T: list                 # T_1, T_3, T_4, T_5, T_6 (points)
    x: int
    l: list
    r: list
    t: int
    tau_x: int
    mu: int
    transcript_log: list = field(default_factory=list)  # (label, bytes) appended, in order
    verify: dict = field(default_factory=dict)


class Engine:
    """The group operations of the flow at the reference's call sites, and
    its transcript.  This default is the oracle's own (pure Python); a test
    substitutes the product's C ABI to check it call site by call site."""

    def __init__(self):
        self.B = self.Bb = self.G = self.H = None

    def set_gens(self, B, Bb, G, H):
        self.B, self.Bb, self.G, self.H = B, Bb, G, H

    def msm(self, scalars, points):  # vartime_multiscalar_mul
        return r255.msm_pippenger([s % L for s in scalars], list(points))

    def commit(self, v, blind):  # PedersenGens::commit (weights.rs:60) and the T_i (2 terms over B, B_blinding)
        return self.msm([v, blind], [self.B, self.Bb])

    def vec_commit(self, blind, a, b=None):  # A_I, A_O, S (circuit_lib.rs:187-229)
        if b is None:
            return self.msm([blind] + list(a), [self.Bb] + self.G[:len(a)])
        return self.msm([blind] + list(a) + list(b), [self.Bb] + self.G[:len(a)] + self.H[:len(b)])

    def transcript(self, label):
        return Transcript(label)


def compat_prove(k: int, seed: int, label: bytes = b"test", engine: Engine | None = None) -> CompatRun:
    """test_first(n = 2k, m = 2k + 1) (lib.rs:160-233) through
    blinding_values, then verify's computations, with the group operations
    and the transcript of `engine` (the oracle's by default)."""
    eng = engine or Engine()
    n, Q, m = 2 * k, 4 * k, 2 * k + 1
    rng = Rng(seed, b"bpperm-compat")
    # lib.rs:161-180: random PedersenGens, the (unused) H_factors challenge,
    # random G and H
    B, Bb = rng.point(), rng.point()
    rng.scalar()  # rand_chal -> H_factors (never reaches create: :190, :194 commented out)
    G = [rng.point() for _ in range(n)]
    H = [rng.point() for _ in range(n)]
    eng.set_gens(B, Bb, G, H)
    # weights.rs:37-56 create_variables: [1..k] ++ shuffle([1..k]) ++ [x = 1]
    perm = fisher_yates(k, rng)
    v = list(range(1, k + 1)) + [p + 1 for p in perm] + [1]
    # weights.rs:58-61 commit_variables: fresh blindings
    V_blind = [rng.scalar() for _ in range(m)]
    V = [eng.commit(vi, bl) for vi, bl in zip(v, V_blind)]
    # lib.rs:188 binds `let (w_r, w_l, w_o, w_v) = create_weights(k);` and
    # passes W_L: w_l, W_R: w_r (:203-204): the reference's W_L is the matrix
    # create_weights builds as w_r (its i >= n rows, weights.rs:153) and its
    # W_R is create_weights' w_l (the i < n rows, :141)
    wr, wl, wo, wv = compat_create_weights(k)
    WL, WR, WO, WV = _transpose(wl), _transpose(wr), _transpose(wo), _transpose(wv)  # Q2
    c = [0] * (Q - 2) + [L - 1, 1]  # weights.rs:26-35 create_constants
    aL, aR, aO = compat_create_a(v)  # Q3
    gamma = [rng.scalar() for _ in range(m)]  # lib.rs:196
    log = []
    tr = eng.transcript(label)

    def append(lab, b):
        log.append((lab, b))
        tr.append_message(lab, b)

    # circuit_lib.rs:139-253 create
    assert len(WL) == n and len(WL[0]) == Q and len(WV) == m
    log.append((b"dom-sep", b"acp v1"))
    log.append((b"n", n.to_bytes(8, "little")))
    tr.arithmetic_domain_sep(n)
    alpha, beta, ro = rng.scalar(), rng.scalar(), rng.scalar()
    A_I = eng.vec_commit(alpha, aL, aR)                   # :187-200
    A_O = eng.vec_commit(beta, aO)                        # :202-210
    s_l = [rng.scalar() for _ in range(n)]                # :213
    s_r = [rng.scalar() for _ in range(n)]                # :214 (rng_2: the same thread RNG)
    S = eng.vec_commit(ro, s_l, s_r)                      # :216-229
    for lab, P in ((b"A_I", A_I), (b"A_O", A_O), (b"S", S)):  # :231-233
        append(lab, r255.encode(P))
    # :135-138 challenge_wit_and_const
    y = tr.challenge_scalar(b"y")
    z = tr.challenge_scalar(b"z")
    # :256-302 compute_per_challenges
    y_n = compat_exp_iter(y, n)                           # Q1
    y_n_inv = [r255.scalar_inv(e) for e in y_n]
    z_q = compat_exp_iter(z, Q)                           # Q1
    z_W_R = vm_mult(z_q, WR)
    l_in = hadamard(y_n_inv, z_W_R)
    z_W_L = vm_mult(z_q, WL)
    sigma = inner(l_in, z_W_L)
    # :304-423 commit_Ts
    zero = [0] * n
    l_x = [zero, [(a + b) % L for a, b in zip(aL, l_in)], list(aO), list(s_l)]
    r_x = [[(a - b) % L for a, b in zip(vm_mult(z_q, WO), y_n)],
           [(a + b) % L for a, b in zip(hadamard(y_n, aR), vm_mult(z_q, WL))],
           zero,
           hadamard(y_n, s_r)]
    t_poly = special_inner_product(l_x, r_x)
    taus, t_vals, T = [], [], []
    for i in (1, 3, 4, 5, 6):
        tau = rng.scalar()
        ti = poly6_eval(t_poly, i)                        # Q4: t(i), not t_i
        Ti = eng.commit(ti, tau)
        taus.append(tau)
        t_vals.append(ti)
        T.append(Ti)
    # appends: T1, T3, then T_3's bytes under "T4" (Q5), T5, T6
    for lab, P in ((b"T1", T[0]), (b"T3", T[1]), (b"T4", T[1]), (b"T5", T[3]), (b"T6", T[4])):
        append(lab, r255.encode(P))
    # :425-432
    x = tr.challenge_scalar(b"x")
    # :434-476 blinding_values
    l = vecpoly3_eval(l_x, x)
    r = vecpoly3_eval(r_x, x)
    t = inner(l, r)
    wvg = inner(z_q, mv_mult(WV, gamma))
    tau_x = 0
    for tau, e in zip(taus, (1, 3, 4, 5, 6)):             # Q6: the x^2 term five times
        tau_x = (tau_x + tau * scalar_exp(x, e) + x * x * wvg) % L
    mu = (alpha * x + beta * scalar_exp(x, 2) + ro * scalar_exp(x, 3)) % L
    append(b"TX", r255.scalar_bytes(tau_x))
    append(b"mu", r255.scalar_bytes(mu))
    # (Q8: "l", "r" as bytevec strings and then "t" -- unpinned bytes, not appended)
    run = CompatRun(k, n, Q, m, B, Bb, G, H, v, V_blind, V, gamma, aL, aR, aO, WL, WR, WO, WV, c, alpha, beta,
                    ro, s_l, s_r, A_I, A_O, S, y, z, y_n, y_n_inv, z_q, z_W_L, z_W_R, l_in, sigma, t_poly, taus,
                    t_vals, T, x, l, r, t, tau_x, mu, log)
    run.verify = compat_verify(run, eng)
    return run


def compat_verify(run: CompatRun, engine: Engine | None = None) -> dict:
    """circuit_lib.rs:478-585 on the prover's state: the group elements it
    forms and the outcome of its two live checks."""
    msm = (engine or Engine()).msm
    x = run.x
    h_ = [msm([yi], [Hi]) for yi, Hi in zip(run.y_n_inv, run.H)]            # :491 (h_i = H_i y^-i, Q1 powers)
    weights_L = msm(run.z_W_L, h_)                                          # :498-501
    weights_R = msm(run.l_in, run.G)                                        # :504-507
    weights_O = msm(vm_mult(run.z_q, run.WO), h_)                           # :509-512
    t_ok = run.t == inner(run.l, run.r)                                     # :518-520
    g_exp = scalar_exp(x, 2) * (inner(run.z_q, run.c) + run.sigma) % L      # :521
    v_exp = [scalar_exp(x, 2) * e % L for e in vm_mult(run.z_q, run.WV)]    # :522
    t_exp = [x] + [scalar_exp(x, i) for i in range(3, 7)]                   # :523
    cand = msm([g_exp] + v_exp + t_exp, [run.B] + run.V + run.T)            # :525-533
    gt_htau = msm([run.t, run.tau_x], [run.B, run.Bb])                      # :535-538
    tau_ok = r255.equal(gt_htau, cand)                                      # :541-544
    P = msm([x, scalar_exp(x, 2)] + [(-e) % L for e in run.y_n] + [x, x, 1, scalar_exp(x, 3)],
            [run.A_I, run.A_O] + h_ + [weights_L, weights_R, weights_O, run.S])   # :551-565
    cand_P = msm([run.mu] + run.l + run.r, [run.Bb] + run.G + run.H)       # :568-575
    return {"h_": h_, "weights_L": weights_L, "weights_R": weights_R, "weights_O": weights_O,
            "t_ok": t_ok, "gt_htau_cand": cand, "gt_htau": gt_htau, "tau_ok": tau_ok,
            "P": P, "cand_P": cand_P, "P_ok": r255.equal(P, cand_P),
            # the reference returns Err at the first failing live check; Q7
            # leaves P == cand_P unchecked
            "result": "ok" if (t_ok and tau_ok) else ("Err(t)" if not t_ok else "Err(tau)")}
