"""ORACLE — test infrastructure only.

CPU restatement of the reference's kernel semantics, used as the checker by
``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py``. Nothing in ``pystencils_autodiff_amd`` imports, links or runs
anything from here; the product path fails loudly when its HIP extension is
missing instead of falling back to this code.

* ``evaluate.py`` — float64 NumPy evaluation of an assignment collection with
  the semantics of pystencils kernels as the reference builds them
  (``_autodiff.py:479-542``, ``transformations.py:12-36``): zero padding for
  ``boundary_handling='zeros'``, interior-only writes (``required_ghost_layers``
  border) for ``None``; statements in order, subexpressions first.
* ``stencils.py`` — the BASELINE.json workloads written out by hand, forward
  AND adjoint, independent of the symbolic AD core (the adjoints are derived on
  paper from TF-MAD, ``_autodiff.py:104-109``).
* ``stencil_ref.c`` (+ ``Makefile``) — the same workloads as the plain C loop
  nests pystencils' CPU backend generates (``generate_c(dialect='c')``,
  ``printer.py:73-75``), optionally OpenMP-parallel (``cpu_openmp``,
  ``_autodiff.py:487-489``); timed as the CPU baseline in ``bench.py``.

Pinning: the reference cannot run here (pystencils is
an un-vendored dependency). The symbolic derivation is pinned by the
reference's own known-answer strings (``tests/test_autodiff.py:21,46``,
``docs/index.rst:71-78``); adjoint correctness by the reference's gradcheck
tests (``tests/test_tfmad.py:186-285``) and the dot-product identity;
the numeric kernel evaluation has no reference vectors to pin against.
"""
