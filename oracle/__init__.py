"""TEST INFRASTRUCTURE ONLY — the parity oracle for tmhpvsim_amd.

Nothing in the product package (`tmhpvsim_amd/`) imports, links or executes
anything under `oracle/`.  Only `tests/`, `__graft_entry__.smoke()` and the
`cpu_baseline` leg of `bench.py` use it, and only as the checker.

Contents
--------
philox.py       numpy restatement of Random123 Philox4x32-10 + the 52-bit
                uniform conversion used by every uniform stream (KAT-pinned).
variates.py     the harness' inverse-CDF variate mapping (one uniform → one
                variate), restated from scipy's `ndtri`/`gammaincinv`/`stdtrit`
                call sites.
ref_harness.py  injected-uniform harness around the *imported* reference
                (`/root/reference`, build container only) that generates the
                golden fixtures in `tests/golden/`.
tmh_oracle.c    plain-C restatement of the reference hot path
                (clearskyindexmodel.py, cloud_cover_binary.py,
                cloud_cover_hourly.py sampling, pvmodel.py PV chain,
                metersim.get_meter_value, pvsim residual) — the CPU checker
                and the bench's CPU baseline (`kind: "port"`).
oracle.py       ctypes wrapper for the compiled `liboracle.so`.
"""
