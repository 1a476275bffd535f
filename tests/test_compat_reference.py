"""Pins the oracle's reading of the reference's deterministic code (compat
mode: the behaviour as written, defects included).

Expected values are derived by hand from the Rust source:
* util.rs:63-65,138-157 `exp_iter` / `ScalarExp::next`: state (x=1,
  next=x); each call yields next, then next *= x_state, x_state = yielded.
  Exponents 1, 1, 2, 3, 5, 8, ... (Fibonacci; defect Q1).
* weights.rs:130-204 `create_weights`: dense Q x n matrices (Q = 4k rows,
  n = 2k columns; defect Q2 — `create` expects n x Q).
* weights.rs:63-113 `create_a`: the gate chains with a_L[n-1] = a_O[offset]
  + a_O[n-2] (offset = (n-1)/2, the second chain's first gate; defect Q3) and
  a_O[n-1] = a_L[n-1]^2.
"""
from oracle import bulletproofs as bp
from oracle.merlin import Rng

L = bp.L


def test_exp_iter_fibonacci_exponents():
    # x, x, x^2, x^3, x^5, x^8, x^13
    assert bp.compat_exp_iter(2, 7) == [2, 2, 4, 8, 32, 256, 8192]
    assert bp.compat_exp_iter(3, 6) == [3, 3, 9, 27, 243, 6561]
    x = 0x1234567890ABCDEF
    assert bp.compat_exp_iter(x, 6) == [pow(x, e, L) for e in (1, 1, 2, 3, 5, 8)]


def test_create_weights_k4_by_hand():
    k, n, Q = 4, 8, 16
    wl, wr, wo, wv = bp.compat_create_weights(k)
    assert (len(wl), len(wl[0]), len(wv[0])) == (Q, n, n + 1)  # Q x n (not n x Q)

    def nz(M):
        return {(q, i): v for q, row in enumerate(M) for i, v in enumerate(row) if v}

    assert nz(wl) == {(i, i): 1 for i in range(n)}
    assert nz(wr) == {(i, i - n): 1 for i in range(n, Q)}
    # w_o[i][i-1] = 1 for 0 < i < n, i != k/2 + 1 = 3; then w_o[n-1][k-1] = 1
    assert nz(wo) == {**{(i, i - 1): 1 for i in (1, 2, 4, 5, 6, 7)}, (7, 3): 1}
    want_v = {(0, 8): L - 1, (0, 0): 1, (3, 8): L - 1, (3, 4): 1}
    for i in range(n, Q - 2):  # rows 8..13: -x and v[i-n+1] (i < n+3) or v[i-n+2]
        want_v[(i, 8)] = L - 1
        want_v[(i, i - n + 1 if i < n + 3 else i - n + 2)] = 1
    assert nz(wv) == want_v


def test_create_a_k4_by_hand():
    # v = [1, 2, 3, 4, pi = 2, 1, 4, 3, x = 10]; n = 8, offset = 3
    aL, aR, aO = bp.compat_create_a([1, 2, 3, 4, 2, 1, 4, 3, 10])
    m = lambda v: v % L  # noqa: E731
    assert aR == [m(-8), m(-7), m(-6), m(-9), m(-6), m(-7), m(-1), 1]
    assert aL == [m(-9), 72, m(-504), m(-8), 72, m(-432), 3024, m(72 - 3024)]
    assert aO == [72, m(-504), 3024, 72, m(-432), 3024, m(-3024), (72 - 3024) ** 2 % L]
    # both chains end at the same product (a permutation), but the
    # combination gate reads a_O[offset] = 72, not the first chain's end 3024
    assert aO[2] == aO[5] == 3024 and aL[7] != 0


def _violations(k, perm, x=1, bind_as_lib_rs=True):
    """Violated linear / multiplication constraints of the reference's
    witness.  lib.rs:188 binds `let (w_r, w_l, w_o, w_v) = create_weights(k)`
    and passes W_L: w_l, W_R: w_r (:203-204), so the reference's W_L is
    create_weights' SECOND return; bind_as_lib_rs=False reads the matrices
    in create_weights' own order instead."""
    v = list(range(1, k + 1)) + [p + 1 for p in perm] + [x]
    aL, aR, aO = bp.compat_create_a(v)
    first, second, wo, wv = bp.compat_create_weights(k)
    wl, wr = (second, first) if bind_as_lib_rs else (first, second)
    Q, n = 4 * k, 2 * k
    c = [0] * (Q - 2) + [L - 1, 1]  # create_constants (weights.rs:26-36)
    held = []
    for q in range(Q):
        lhs = sum(wl[q][i] * aL[i] + wr[q][i] * aR[i] + wo[q][i] * aO[i] for i in range(n)) % L
        rhs = (sum(wv[q][j] * v[j] for j in range(n + 1)) + c[q]) % L
        if lhs == rhs:
            held.append(q)
    mul = sum((aL[i] * aR[i] - aO[i]) % L != 0 for i in range(n))
    return Q - len(held), mul, held


def test_reference_witness_violates_its_constraints_k52():
    """SURVEY.md §2.2 Q3, re-derived under the reference's actual binding
    (lib.rs:188, 203-204): with x = 1 (weights.rs:50) every 52-card witness
    violates 207 of the 208 linear constraints -- only row k/2 + 1 = 27
    (create_weights' special a_L row, weights.rs:144-150) holds -- and the
    last multiplication gate.  Read in create_weights' own order (the
    binding SURVEY Q3 assumed) the same witnesses violate 49-100 rows."""
    rng = Rng(3, b"compat")
    for _ in range(6):
        perm = bp.fisher_yates(52, rng)
        lin, mul, held = _violations(52, perm)
        assert (lin, mul, held) == (207, 1, [27])
        lin_cw, mul_cw, _ = _violations(52, perm, bind_as_lib_rs=False)
        assert 49 <= lin_cw <= 100 and mul_cw == 1


def test_compat_restatement_binds_weights_as_lib_rs():
    """oracle/compat.py's W_L is create_weights' w_r (ones in rows i >= n,
    weights.rs:153) and its W_R is create_weights' w_l (ones in rows i < n,
    weights.rs:141), both transposed for create() (Q2)."""
    from oracle import compat
    k = 3
    run = compat.compat_prove(k, 0)
    n, Q = 2 * k, 4 * k
    first, second, _, _ = bp.compat_create_weights(k)
    assert run.WL == [[second[q][i] for q in range(Q)] for i in range(n)]
    assert run.WR == [[first[q][i] for q in range(Q)] for i in range(n)]
    assert all(run.WL[i][q] == (1 if q == i + n else 0) for i in range(n) for q in range(Q))
    assert all(run.WR[i][q] == (1 if q == i else 0) for i in range(n) for q in range(Q))
