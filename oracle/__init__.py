"""CPU oracle for the rlmd_amd hot path — TEST INFRASTRUCTURE ONLY.

A restatement of the reference's algorithms (majidsina/rlmd, cited file:line
in each module) in NumPy / PyTorch-CPU, used by tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg as the CHECKER.  The product path
(rlmd_amd/librlmd_amd.so) never imports, links or calls anything here.

Pinning: every module is checked against golden vectors produced by the
reference itself (tests/golden/make_golden.py, run in the build container with
the reference importable) — see tests/test_oracle_golden.py.
"""
