"""ORACLE -- TEST INFRASTRUCTURE ONLY.

A CPU restatement (torch-CPU ops, float arithmetic exactly as the reference
performs it) of the Aris-ma/AllreduceTopK comm-hook codecs:

* ``oracle.arctopk`` -- ARC-TopK (comm_hooks/group_topk_hook_no_reshape.py)
* ``oracle.sparse``  -- TopK / RandK baselines (comm_hooks/sparse_hook.py,
  comm_hooks/sparse_hook_c4.py)

It is the *checker*, never the product: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import it.
The shipped hooks in ``allreducetopk_amd`` run the HIP kernels of
``libarctopk.so`` and fail loudly when that library is missing.

Parity pinning: the restatement is checked bit-for-bit against golden vectors
produced by running the reference hooks themselves in the build container
(``tests/golden/make_golden.py`` -> ``tests/golden/*.npz``; test
``tests/test_oracle_golden.py``).  The reference ships no tests or fixtures of
its own for this path, so those generated vectors are
the pin.
"""
