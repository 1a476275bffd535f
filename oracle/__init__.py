"""CPU oracle for the bulletproof-perm hot path — TEST INFRASTRUCTURE ONLY.

This package is a from-the-spec restatement of the arithmetic the reference
(`ercembu/bulletproof-perm`, Rust) delegates to third-party crates that are not
vendored under /root/reference (pins from `bp-perm/Cargo.lock`):

  * curve25519-dalek-ng 4.1.1 — field GF(2^255-19), Scalar mod l, Edwards and
    Ristretto group, `vartime_multiscalar_mul` (Straus / Pippenger dispatch);
  * merlin 3.0.0 — STROBE-128 / Keccak-f[1600] Fiat-Shamir transcript;
  * bulletproofs 4.0.0 — PedersenGens, BulletproofGens (GeneratorsChain),
    InnerProductProof create / verify.

`compat.py` restates the reference's own driver (test_first) as written,
defects included (compat mode; test-only).

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg
may import anything from here, and only as the checker.  The product path
(`bulletproof-perm_amd/`) never imports, links or executes this package.

Parity pins (see DESIGN.md "Oracle"): RFC 9496 ristretto255 test vectors,
the Merlin "simple transcript" KAT, `PedersenGens::default().B_blinding`, and an
OpenSSL Ed25519 public-key cross-check (same curve).  The reference's own tests
pin no numeric result, so the protocol-level pieces that no KAT
covers (GeneratorsChain label bytes, IPA transcript labels) are "parity
unpinned" beyond self-consistency (prove -> verify).
"""
