"""Compat mode ("both compat and sound modes"):
the reference's test_first (lib.rs:160-233) restated AS WRITTEN in
oracle/compat.py, defects included.  These CPU tests check the
restatement's internal algebra and its defects against the cited lines;
tests/test_gpu_compat.py runs the same flow's group operations through the
product's C ABI.  Parity unpinned (thread_rng; the reference holds no
fixtures): compat_k3_seed0.json pins the restatement against drift."""
import json
from pathlib import Path

import pytest

from oracle import compat
from oracle import ristretto as r255

L = r255.L
GOLDEN = Path(__file__).resolve().parent / "golden" / "compat_k3_seed0.json"


@pytest.fixture(scope="module", params=[3, 52])
def run(request):
    return compat.compat_prove(request.param, 0)


def test_verify_fails_where_the_reference_says(run):
    # circuit_lib.rs:518 (t == <l, r>) passes; :541-543 "IT ALREADY FAILS HERE"
    assert run.verify["t_ok"] and not run.verify["tau_ok"]
    assert run.verify["result"] == "Err(tau)"
    assert not run.verify["P_ok"]  # Q7: unchecked, and it would fail too


def test_t_polynomial_is_the_inner_product_of_l_and_r(run):
    # poly.rs special_inner_product / Poly6::eval against <l(x), r(x)>
    assert run.t == compat.poly6_eval(run.t_poly, run.x)


def test_q1_fibonacci_powers(run):
    y = run.y
    e = [1, 1]
    while len(e) < run.n:
        e.append(e[-1] + e[-2])
    assert run.y_n == [pow(y, k, L) for k in e[:run.n]]
    assert len(run.z_q) == run.Q


def test_q4_T_commits_to_values_not_coefficients(run):
    for i, ti in zip((1, 3, 4, 5, 6), run.t_vals):
        assert ti == compat.poly6_eval(run.t_poly, i)
    # the coefficient t_1 is not t(1) (t(1) = t_1 + ... + t_6)
    assert run.t_vals[0] != run.t_poly[0]


def test_q5_T4_label_carries_T3(run):
    log = dict(run.transcript_log)
    assert log[b"T4"] == r255.encode(run.T[1]) != r255.encode(run.T[2])
    labels = [lab for lab, _ in run.transcript_log]
    assert labels == [b"dom-sep", b"n", b"A_I", b"A_O", b"S", b"T1", b"T3", b"T4", b"T5", b"T6", b"TX", b"mu"]


def test_q6_gamma_term_five_times(run):
    wvg = compat.inner(run.z_q, compat.mv_mult(run.WV, run.gamma))
    taus = sum(t * pow(run.x, e, L) for t, e in zip(run.taus, (1, 3, 4, 5, 6))) % L
    assert (run.tau_x - taus) % L == 5 * run.x * run.x * wvg % L


def test_q2_shapes_and_commit_blindings(run):
    assert len(run.WL) == run.n and len(run.WL[0]) == run.Q  # transposed for create()
    assert len(run.WV) == run.m == len(run.gamma) == len(run.V)
    assert run.V_blind != run.gamma  # V's blindings are not the gamma of tau_x


def test_golden_k3():
    import importlib.util
    spec = importlib.util.spec_from_file_location("mk", GOLDEN.parent / "make_compat_golden.py")
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    assert mk.summary(compat.compat_prove(3, 0)) == json.loads(GOLDEN.read_text())
