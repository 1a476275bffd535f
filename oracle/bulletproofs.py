"""Inner-product argument + permutation arithmetic-circuit proof — TEST ONLY.

Spec restatement of what the reference builds on (SURVEY.md App. B2 and
§2.2), in the plainest form, as the checker for the HIP product path:

  ipa_create / ipa_verify   bulletproofs 4.0.0 InnerProductProof::create /
                            verify (folding form: G, H folded with 2-term MSMs
                            each round).  The reference never runs an IPA —
                            it sends l, r in the clear (circuit_lib.rs:466-467,
                            518); its hook fields ACEssentials.G_factors /
                            H_factors (circuit_lib.rs:62-63) are for this.
  perm_circuit              the permutation circuit of weights.rs:26-204 /
                            create_a weights.rs:63-113, in SOUND form: the
                            Q3 fix (chain-1 end a_O[k-2]), a_O[n-1] = a_L*a_R,
                            a random challenge x bound to v_{2k}.
  ac_prove / ac_verify      ArithmeticCircuitProof (circuit_lib.rs:139-585)
                            in SOUND form (Bulletproofs paper, Protocol 3):
                            standard powers (Q1), non-transposed W (Q2),
                            T_i commit to coefficients t_i (Q4), tau_x adds
                            x^2<z,W_V gamma> once (Q6), T4 appended as T4
                            (Q5), V bound by the transcript (Q9), a proof
                            object instead of shared prover state (Q10), IPA
                            instead of clear l, r (Q8).
  compat_*                  the reference's deterministic pieces AS WRITTEN
                            (Fibonacci exp_iter Q1, create_a Q3, create_weights
                            Q2 shape) — documented behaviour, not used by the
                            product.

Parity status: the primitives under these (ristretto255, Merlin) are
KAT-pinned; GeneratorsChain label bytes and the IPA transcript labels are
recalled from bulletproofs 4.0.0 and "parity unpinned" beyond prove->verify
self-consistency.
"""
from __future__ import annotations

from dataclasses import dataclass, field

from . import ristretto as r255
from .merlin import Rng, Transcript, bulletproof_gens, indexed_scalar, pedersen_gens_default

L = r255.L


def inner(a, b):
    return sum(x * y for x, y in zip(a, b)) % L


def powers(x, n):
    out, c = [], 1
    for _ in range(n):
        out.append(c)
        c = c * x % L
    return out


def enc(p):
    return r255.encode(p)


def msm(scalars, points):
    return r255.msm_pippenger([s % L for s in scalars], points, 4 if len(points) < 8 else 6)


# =========================================================================== IPA
@dataclass
class IPAProof:
    L: list
    R: list
    a: int
    b: int

    def to_bytes(self) -> bytes:
        out = b""
        for l_, r_ in zip(self.L, self.R):
            out += l_ + r_
        return out + r255.scalar_bytes(self.a) + r255.scalar_bytes(self.b)


def ipa_create(tr: Transcript, Q, G_factors, H_factors, G, H, a, b) -> IPAProof:
    """bulletproofs 4.0.0 InnerProductProof::create."""
    n = len(G)
    assert n == len(H) == len(a) == len(b) == len(G_factors) == len(H_factors)
    assert n & (n - 1) == 0
    tr.innerproduct_domain_sep(n)
    G, H, a, b = list(G), list(H), list(a), list(b)
    Ls, Rs = [], []
    first = True
    while n != 1:
        n //= 2
        a_L, a_R, b_L, b_R = a[:n], a[n:], b[:n], b[n:]
        G_L, G_R, H_L, H_R = G[:n], G[n:], H[:n], H[n:]
        c_L, c_R = inner(a_L, b_R), inner(a_R, b_L)
        if first:
            gf_lo, gf_hi = G_factors[:n], G_factors[n:]
            hf_lo, hf_hi = H_factors[:n], H_factors[n:]
        else:
            gf_lo = gf_hi = hf_lo = hf_hi = [1] * n
        Lp = msm([x * g for x, g in zip(a_L, gf_hi)] + [x * h for x, h in zip(b_R, hf_lo)] + [c_L],
                 G_R + H_L + [Q])
        Rp = msm([x * g for x, g in zip(a_R, gf_lo)] + [x * h for x, h in zip(b_L, hf_hi)] + [c_R],
                 G_L + H_R + [Q])
        Le, Re = enc(Lp), enc(Rp)
        Ls.append(Le)
        Rs.append(Re)
        tr.append_point(b"L", Le)
        tr.append_point(b"R", Re)
        u = tr.challenge_scalar(b"u")
        ui = r255.scalar_inv(u)
        a = [(a_L[i] * u + ui * a_R[i]) % L for i in range(n)]
        b = [(b_L[i] * ui + u * b_R[i]) % L for i in range(n)]
        G = [msm([ui * gf_lo[i], u * gf_hi[i]], [G_L[i], G_R[i]]) for i in range(n)]
        H = [msm([u * hf_lo[i], ui * hf_hi[i]], [H_L[i], H_R[i]]) for i in range(n)]
        first = False
    return IPAProof(Ls, Rs, a[0], b[0])


def ipa_verification_scalars(proof: IPAProof, n: int, tr: Transcript):
    lg_n = len(proof.L)
    if lg_n >= 32 or n != (1 << lg_n):
        raise ValueError("VerificationError")
    tr.innerproduct_domain_sep(n)
    us = []
    for Le, Re in zip(proof.L, proof.R):
        tr.validate_and_append_point(b"L", Le)
        tr.validate_and_append_point(b"R", Re)
        us.append(tr.challenge_scalar(b"u"))
    uinv = [r255.scalar_inv(u) for u in us]
    allinv = 1
    for x in uinv:
        allinv = allinv * x % L
    u_sq = [u * u % L for u in us]
    uinv_sq = [x * x % L for x in uinv]
    s = [allinv]
    for i in range(1, n):
        lg_i = i.bit_length() - 1
        k = 1 << lg_i
        s.append(s[i - k] * u_sq[lg_n - 1 - lg_i] % L)
    return u_sq, uinv_sq, s


def ipa_verify_msm_terms(proof, n, tr, G_factors, H_factors, Q, G, H):
    """(scalars, points) whose MSM equals expect_P of bulletproofs' verify."""
    u_sq, uinv_sq, s = ipa_verification_scalars(proof, n, tr)
    a, b = proof.a, proof.b
    sc = [a * b % L]
    pts = [Q]
    sc += [a * s[i] % L * G_factors[i] % L for i in range(n)]
    pts += list(G)
    sc += [b * s[n - 1 - i] % L * H_factors[i] % L for i in range(n)]
    pts += list(H)
    sc += [(-x) % L for x in u_sq] + [(-x) % L for x in uinv_sq]
    pts += [r255.decode(x) for x in proof.L] + [r255.decode(x) for x in proof.R]
    return sc, pts


def ipa_verify(proof, n, tr, G_factors, H_factors, P, Q, G, H) -> bool:
    sc, pts = ipa_verify_msm_terms(proof, n, tr, G_factors, H_factors, Q, G, H)
    return r255.equal(msm(sc, pts), P)


# ====================================================== permutation circuit
@dataclass
class Circuit:
    k: int
    n: int            # gates = 2k
    n_p: int          # padded to a power of two (IPA length)
    Q: int            # linear constraints = 4k + 2
    m: int            # committed values = 2k + 1
    WL: list = field(default_factory=list)   # sparse rows: list of (q, col, val)
    WR: list = field(default_factory=list)
    WO: list = field(default_factory=list)
    WV: list = field(default_factory=list)
    c: list = field(default_factory=list)    # dense length Q; c[Q-1] = -x set per proof


def perm_circuit(k: int) -> Circuit:
    """Sound-mode weights for the reference's two product chains
    (weights.rs:63-113 shape): prod_i (v_i - x) == prod_i (v'_i - x)."""
    assert k >= 2
    n = 2 * k
    n_p = 1
    while n_p < n:
        n_p *= 2
    Qn = 4 * k + 2
    C = Circuit(k, n, n_p, Qn, 2 * k + 1)
    X = 2 * k  # column of the committed challenge x in v
    neg1 = L - 1
    C.c = [0] * Qn
    # a_L rows (q = g)
    for g in range(n):
        C.WL.append((g, g, 1))
        if g == 0:
            C.WV += [(g, 0, 1), (g, X, neg1)]
        elif g == k - 1:
            C.WV += [(g, k, 1), (g, X, neg1)]
        elif g == 2 * k - 1:
            C.WO += [(g, k - 2, neg1), (g, 2 * k - 2, neg1)]
        else:
            C.WO.append((g, g - 1, neg1))
    # a_R rows (q = n + g)
    for g in range(n):
        q = n + g
        C.WR.append((q, g, 1))
        if g <= k - 2:
            C.WV += [(q, g + 1, 1), (q, X, neg1)]
        elif g <= 2 * k - 3:
            C.WV += [(q, g + 2, 1), (q, X, neg1)]
        elif g == 2 * k - 2:
            C.c[q] = neg1
        else:
            C.c[q] = 1
    C.WO.append((4 * k, 2 * k - 1, 1))       # a_O[n-1] = 0
    C.WV.append((4 * k + 1, X, 1))           # v_2k + c = 0, c = -x
    return C


def perm_witness(k: int, perm, x: int):
    """v = [1..k, pi(1..k), x]; gate values for the two chains (sound
    create_a: a_L[n-1] = a_O[k-2] + a_O[n-2], a_O = a_L * a_R)."""
    v = list(range(1, k + 1)) + [p + 1 for p in perm] + [x]
    n = 2 * k
    aL, aR, aO = [0] * n, [0] * n, [0] * n
    for g in range(k - 1):  # chain A: gates 0..k-2
        aL[g] = (v[0] - x) % L if g == 0 else aO[g - 1]
        aR[g] = (v[g + 1] - x) % L
        aO[g] = aL[g] * aR[g] % L
    for g in range(k - 1, 2 * k - 2):  # chain B: gates k-1..2k-3
        aL[g] = (v[k] - x) % L if g == k - 1 else aO[g - 1]
        aR[g] = (v[g + 2] - x) % L
        aO[g] = aL[g] * aR[g] % L
    g = 2 * k - 2
    aL[g], aR[g] = aO[2 * k - 3], L - 1
    aO[g] = aL[g] * aR[g] % L
    g = 2 * k - 1
    aL[g], aR[g] = (aO[k - 2] + aO[2 * k - 2]) % L, 1
    aO[g] = aL[g] * aR[g] % L
    return [x % L for x in v], aL, aR, aO


def mat_vec_rows(Wsparse, z_q, ncols):
    """(z^Q)^T W as a length-ncols vector (sparse)."""
    out = [0] * ncols
    for q, col, val in Wsparse:
        out[col] = (out[col] + z_q[q] * val) % L
    return out


def check_constraints(C: Circuit, v, aL, aR, aO, x):
    c = list(C.c)
    c[C.Q - 1] = (-x) % L
    lhs = [0] * C.Q
    rhs = list(c)
    for q, col, val in C.WL:
        lhs[q] = (lhs[q] + val * aL[col]) % L
    for q, col, val in C.WR:
        lhs[q] = (lhs[q] + val * aR[col]) % L
    for q, col, val in C.WO:
        lhs[q] = (lhs[q] + val * aO[col]) % L
    for q, col, val in C.WV:
        rhs[q] = (rhs[q] + val * v[col]) % L
    return [q for q in range(C.Q) if lhs[q] != rhs[q]]


def fisher_yates(k: int, rng: Rng):
    p = list(range(k))
    for i in range(k - 1, 0, -1):
        j = int.from_bytes(rng.bytes(8), "little") % (i + 1)
        p[i], p[j] = p[j], p[i]
    return p


@dataclass
class PermProof:
    V: list
    A_I: bytes
    A_O: bytes
    S: bytes
    T: list           # T1, T3, T4, T5, T6
    tau_x: int
    mu: int
    t_hat: int
    ipa: IPAProof

    def to_bytes(self) -> bytes:
        out = self.A_I + self.A_O + self.S + b"".join(self.T)
        out += r255.scalar_bytes(self.tau_x) + r255.scalar_bytes(self.mu) + r255.scalar_bytes(self.t_hat)
        return out + self.ipa.to_bytes()


def _vecpoly_eval(coeffs, x):
    """coeffs: list of vectors [c0, c1, c2, c3] -> sum c_i x^i"""
    n = len(coeffs[0])
    return [(coeffs[0][i] + x * (coeffs[1][i] + x * (coeffs[2][i] + x * coeffs[3][i]))) % L for i in range(n)]


def ac_prove(k: int, seed: int, gens=None, label: bytes = b"bp-perm"):
    """Sound-mode arithmetic-circuit proof for a k-card permutation.  pi from
    the stream Rng(seed, "bpperm-prove") (Fisher-Yates, one u64 per step), the
    blinding scalars by index (indexed_scalar)."""
    rng = Rng(seed, b"bpperm-prove")
    C = perm_circuit(k)
    n, n_p, m = C.n, C.n_p, C.m
    if gens is None:
        gens = bulletproof_gens(n_p)
    G, H = gens
    g, h = pedersen_gens_default()
    perm = fisher_yates(k, rng)
    # scalar draws by index: gamma[m], alpha, beta, rho, s_L[n_p], s_R[n_p], tau[5]
    S = [indexed_scalar(seed, j) for j in range(m + 3 + 2 * n_p + 5)]
    gamma = S[:m]
    alpha, beta, rho = S[m], S[m + 1], S[m + 2]
    sL = S[m + 3: m + 3 + n_p]
    sR = S[m + 3 + n_p: m + 3 + 2 * n_p]
    taus = S[m + 3 + 2 * n_p:]

    tr = Transcript(label)
    tr.arithmetic_domain_sep(n_p)
    vals = list(range(1, k + 1)) + [p + 1 for p in perm]
    V = []
    for j in range(2 * k):
        V.append(enc(msm([vals[j], gamma[j]], [g, h])))
        tr.append_point(b"V", V[-1])
    x_perm = tr.challenge_scalar(b"x_perm")
    V.append(enc(msm([x_perm, gamma[2 * k]], [g, h])))
    tr.append_point(b"V", V[-1])
    v, aL, aR, aO = perm_witness(k, perm, x_perm)
    assert not check_constraints(C, v, aL, aR, aO, x_perm)
    pad = [0] * (n_p - n)
    aL, aR, aO = aL + pad, aR + pad, aO + pad

    A_I = enc(msm([alpha] + aL + aR, [h] + G + H))
    A_O = enc(msm([beta] + aO, [h] + G))
    S = enc(msm([rho] + sL + sR, [h] + G + H))
    for lab, P in ((b"A_I", A_I), (b"A_O", A_O), (b"S", S)):
        tr.append_point(lab, P)
    y = tr.challenge_scalar(b"y")
    z = tr.challenge_scalar(b"z")
    y_n = powers(y, n_p)
    yinv = r255.scalar_inv(y)
    y_inv_n = powers(yinv, n_p)
    z_q = powers(z, C.Q + 1)[1:]
    zWL = mat_vec_rows(C.WL, z_q, n_p)
    zWR = mat_vec_rows(C.WR, z_q, n_p)
    zWO = mat_vec_rows(C.WO, z_q, n_p)
    zWV = mat_vec_rows(C.WV, z_q, m)
    c = list(C.c)
    c[C.Q - 1] = (-x_perm) % L

    l_poly = [[0] * n_p,
              [(aL[i] + y_inv_n[i] * zWR[i]) % L for i in range(n_p)],
              list(aO),
              list(sL)]
    r_poly = [[(zWO[i] - y_n[i]) % L for i in range(n_p)],
              [(y_n[i] * aR[i] + zWL[i]) % L for i in range(n_p)],
              [0] * n_p,
              [y_n[i] * sR[i] % L for i in range(n_p)]]
    t = [0] * 7
    for i in range(4):
        for j in range(4):
            t[i + j] = (t[i + j] + inner(l_poly[i], r_poly[j])) % L
    delta = inner([y_inv_n[i] * zWR[i] % L for i in range(n_p)], zWL)
    assert t[2] == (inner(z_q, [(sum(val * v[col] for (qq, col, val) in C.WV if qq == q) + c[q]) % L
                                for q in range(C.Q)]) + delta) % L
    T = []
    for lab, idx, tau in zip((b"T1", b"T3", b"T4", b"T5", b"T6"), (1, 3, 4, 5, 6), taus):
        T.append(enc(msm([t[idx], tau], [g, h])))
        tr.append_point(lab, T[-1])
    x = tr.challenge_scalar(b"x")
    xp = powers(x, 7)
    tau_x = (sum(tau * xp[i] for tau, i in zip(taus, (1, 3, 4, 5, 6))) + xp[2] * inner(zWV, gamma)) % L
    mu = (alpha * x + beta * xp[2] + rho * xp[3]) % L
    l = _vecpoly_eval(l_poly, x)
    r = _vecpoly_eval(r_poly, x)
    t_hat = inner(l, r)
    assert t_hat == sum(t[i] * xp[i] for i in range(7)) % L
    tr.append_scalar(b"TX", tau_x)
    tr.append_scalar(b"mu", mu)
    tr.append_scalar(b"t", t_hat)
    w = tr.challenge_scalar(b"w")
    Q = r255.ed_mul(w, g)
    ipa = ipa_create(tr, Q, [1] * n_p, y_inv_n, G, H, l, r)
    return PermProof(V, A_I, A_O, S, T, tau_x, mu, t_hat, ipa), perm


def ac_verify_msm_terms(k: int, proof: PermProof, gens=None, label: bytes = b"bp-perm"):
    """Returns (t_check, ipa_check): two (scalars, points) lists, each of
    which must sum to the identity for a valid proof."""
    C = perm_circuit(k)
    n_p, m = C.n_p, C.m
    if gens is None:
        gens = bulletproof_gens(n_p)
    G, H = gens
    g, h = pedersen_gens_default()
    if len(proof.V) != m:
        raise ValueError("VerificationError: V count")
    tr = Transcript(label)
    tr.arithmetic_domain_sep(n_p)
    for j in range(2 * k):
        tr.append_point(b"V", proof.V[j])
    x_perm = tr.challenge_scalar(b"x_perm")
    tr.append_point(b"V", proof.V[2 * k])
    for lab, P in ((b"A_I", proof.A_I), (b"A_O", proof.A_O), (b"S", proof.S)):
        tr.validate_and_append_point(lab, P)
    y = tr.challenge_scalar(b"y")
    z = tr.challenge_scalar(b"z")
    for lab, P in zip((b"T1", b"T3", b"T4", b"T5", b"T6"), proof.T):
        tr.validate_and_append_point(lab, P)
    x = tr.challenge_scalar(b"x")
    tr.append_scalar(b"TX", proof.tau_x)
    tr.append_scalar(b"mu", proof.mu)
    tr.append_scalar(b"t", proof.t_hat)
    w = tr.challenge_scalar(b"w")
    xp = powers(x, 7)
    y_n = powers(y, n_p)
    y_inv_n = powers(r255.scalar_inv(y), n_p)
    z_q = powers(z, C.Q + 1)[1:]
    zWL = mat_vec_rows(C.WL, z_q, n_p)
    zWR = mat_vec_rows(C.WR, z_q, n_p)
    zWO = mat_vec_rows(C.WO, z_q, n_p)
    zWV = mat_vec_rows(C.WV, z_q, m)
    c = list(C.c)
    c[C.Q - 1] = (-x_perm) % L
    delta = inner([y_inv_n[i] * zWR[i] % L for i in range(n_p)], zWL)
    # t check: t_hat g + tau_x h - x^2 (delta + <z,c>) g - x^2 zWV.V - sum x^i T_i == 0
    Vp = [r255.decode(e) for e in proof.V]
    Tp = [r255.decode(e) for e in proof.T]
    t_sc = [(proof.t_hat - xp[2] * (delta + inner(z_q, c))) % L, proof.tau_x]
    t_sc += [(-xp[2] * zWV[j]) % L for j in range(m)]
    t_sc += [(-xp[i]) % L for i in (1, 3, 4, 5, 6)]
    t_pts = [g, h] + Vp + Tp
    # IPA check: P' = x A_I + x^2 A_O + x^3 S - mu h + <x y^-n zWR, G>
    #           + <y^-n (x zWL + zWO) - 1, H> + t_hat w g;  expect_P - P' == 0
    Q = r255.ed_mul(w, g)
    ipa_sc, ipa_pts = ipa_verify_msm_terms(proof.ipa, n_p, tr, [1] * n_p, y_inv_n, Q, G, H)
    # subtract P'
    Pp_sc = [(-x) % L, (-xp[2]) % L, (-xp[3]) % L, proof.mu, (-proof.t_hat * w) % L]
    Pp_pts = [r255.decode(proof.A_I), r255.decode(proof.A_O), r255.decode(proof.S), h, g]
    Pp_sc += [(-x * y_inv_n[i] * zWR[i]) % L for i in range(n_p)]
    Pp_pts += list(G)
    Pp_sc += [(-(y_inv_n[i] * (x * zWL[i] + zWO[i]) - 1)) % L for i in range(n_p)]
    Pp_pts += list(H)
    return (t_sc, t_pts), (ipa_sc + Pp_sc, ipa_pts + Pp_pts)


def ac_verify(k: int, proof: PermProof, gens=None, label: bytes = b"bp-perm") -> bool:
    try:
        (ts, tp), (is_, ip) = ac_verify_msm_terms(k, proof, gens, label)
    except (ValueError, r255.DecodeError):
        return False
    ident = r255.IDENTITY
    return r255.equal(msm(ts, tp), ident) and r255.equal(msm(is_, ip), ident)


# ============================================ reference behaviour as written
def compat_exp_iter(x, n):
    """util.rs:63-65,138-157 ScalarExp::next as written: yields x, x, x^2,
    x^3, x^5, x^8, ... (Fibonacci exponents; defect Q1)."""
    out = []
    cur, nxt = 1, x % L
    for _ in range(n):
        e = nxt
        nxt = nxt * cur % L
        cur = e
        out.append(e)
    return out


def compat_create_a(v):
    """weights.rs:63-113 as written (defect Q3: a_L[n-1] uses a_O[offset];
    a_O[n-1] = a_L^2)."""
    n = len(v) - 1
    aL, aR, aO = [0] * n, [0] * n, [0] * n
    first, second = v[: n // 2], v[n // 2: n]
    x = v[-1]
    off = (n - 1) // 2
    for i in range(len(first) - 1):
        aR[i] = (first[i + 1] - x) % L
        aR[i + off] = (second[i + 1] - x) % L
        if i == 0:
            aL[i] = (first[i] - x) % L
            aL[i + off] = (second[i] - x) % L
        else:
            aL[i] = aO[i - 1]
            aL[i + off] = aO[i + off - 1]
        aO[i] = aL[i] * aR[i] % L
        aO[i + off] = aL[i + off] * aR[i + off] % L
    aL[n - 2] = aO[n - 3]
    aR[n - 2] = L - 1
    aO[n - 2] = aL[n - 2] * aR[n - 2] % L
    aL[n - 1] = (aO[off] + aO[n - 2]) % L
    aR[n - 1] = 1
    aO[n - 1] = aL[n - 1] * aL[n - 1] % L
    return aL, aR, aO


def compat_create_weights(card_count):
    """weights.rs:130-204 as written: dense Q x n matrices (Q = 4k, n = 2k)
    that `create` (circuit_lib.rs:157) expects transposed (defect Q2)."""
    n = card_count * 2
    Qn = n * 2
    wl = [[0] * n for _ in range(Qn)]
    wr = [[0] * n for _ in range(Qn)]
    wo = [[0] * n for _ in range(Qn)]
    wv = [[0] * (n + 1) for _ in range(Qn)]
    for i in range(Qn):
        if i < n:
            wl[i][i] = 1
            if i != (card_count // 2) + 1 and i != 0:
                wo[i][i - 1] = 1
            else:
                wv[i][n] = L - 1
                if i == 0:
                    wv[i][i] = 1
                else:
                    wv[i][i + 1] = 1
        else:
            wr[i][i - n] = 1
            if i < Qn - 2:
                wv[i][n] = L - 1
                if i < n + 3:
                    wv[i][i - n + 1] = 1
                else:
                    wv[i][i - n + 2] = 1
    wo[n - 1][card_count - 1] = 1
    return wl, wr, wo, wv
