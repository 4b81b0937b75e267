"""CPU oracle -- TEST INFRASTRUCTURE ONLY.

This package restates the reference's hot path on the CPU (numpy / scipy /
torch-CPU) so that the HIP product path can be checked against it.  Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import it, and only as the checker / the timed CPU baseline -- never as the
thing measured or shipped.  The product package
``learningsparsepreconditioner4gpu_amd`` must not import this module.

Pinning (see DESIGN.md "Oracle"):

* ``oracle.linalg`` -- CSR assembly with Dirichlet masking, the ext_spai /
  ext_spai_scaled / diagonal preconditioners and the scipy-ordered PCG loop.
  Pinned against the reference itself: ``tests/golden/make_golden.py`` imports
  ``neural_cg.utils.validate`` / ``neural_cg.data`` from /root/reference (with
  import shims for loguru / torch_geometric / typing.override, this container
  only) and records its outputs as ``tests/golden/*.npz``.
* ``oracle.gnn`` -- torch-CPU restatement of ``NodeEdgeProcessing`` with
  PyG 2.6.1 message-passing semantics.  Module structure / parameter names /
  seeded initialisation are pinned against the reference's own constructors;
  the forward arithmetic is **parity unpinned** against PyG (not installed,
  and the reference ships no checkpoint or test vectors).
* The reference's native solver (pymathprim) is unvendored and absent: its
  PCG results are **parity unpinned**; the oracle follows the reference's own
  scipy restatement (``neural_cg/utils/validate.py:163-341``).
"""
