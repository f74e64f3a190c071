"""Oracle: CPU restatements of the reference sBayes hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this package, and only as the checker (or as the timed CPU baseline).
The product path in ``contact_zones_amd`` never imports, links or executes it.

Contents
  lik_numpy.py   numpy restatement of Likelihood.__call__ (sbayes/model.py:145-452)
  sbz_oracle.c   C restatement of the same, numpy pairwise summation order
  oracle_c.py    ctypes wrapper for liboracle.so (built by ``make -C oracle``)
  mh_numpy.py    restatement of the MH step and zone/parameter operators
                 (sbayes/sampling/mcmc_generative.py:282-351, zone_sampling.py:408-933)
                 driven by a recorded draw tape

Pinning: every function here is checked against golden vectors captured from the
reference itself (tests/golden/make_golden.py imports /root/reference in the build
container and writes tests/golden/*.npz); see tests/test_oracle_golden.py.
"""
