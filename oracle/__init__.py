"""CPU oracle for the PDS/APGD hot path -- TEST INFRASTRUCTURE ONLY.

Nothing in ``pycsou_amd`` imports this package.  Only ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` may
use it, and only as the checker / the timed CPU baseline, never as the path
being measured or shipped.

Contents
--------
``oracle.pylops1``
    NumPy/SciPy restatement of the PyLops 1.x operators that pycsou wraps
    (``FirstDerivative``, ``SecondDerivative``, ``Gradient``, ``Laplacian``,
    ``Convolve1D``, ``Convolve2D``).  PyLops is a third-party dependency that
    is absent from ``/root/reference`` (``requirements.txt``: ``pylops >= 1.9.2``;
    the ``N=``/``dir=``/``nodir=`` keywords at ``pycsou/linop/diff.py:128`` and
    ``pycsou/linop/conv.py:163,294`` fix the 1.x API).
``oracle.pycsou_ref``
    NumPy restatement of the reference's own solver / prox / functional code
    (``pycsou/opt/proxalgs.py``, ``pycsou/func/*.py``, ``pycsou/math/prox.py``,
    ``pycsou/core/solver.py``) with the same operation order, temporaries and
    diagnostics semantics.

Pinning
-------
* ``pycsou_ref`` is pinned against golden vectors produced by the *real*
  reference code (imported from ``/root/reference`` in the build container,
  see ``tests/golden/make_golden.py``) -- solver trajectories, diagnostics,
  prox/fenchel values and the reference doctest values.
* ``pylops1.Convolve1D/Convolve2D`` forward are pinned by the reference
  doctests (``pycsou/linop/conv.py:67-73, 209-217``: equality with
  ``scipy.signal.convolve(mode='same')``); adjoints by dot-product tests.
* ``pylops1.FirstDerivative`` forward interior is pinned by
  ``pycsou/linop/diff.py:72-78`` and ``Gradient`` by ``diff.py:814-820``.
  Edge rows (forward last sample, centered ``edge=True`` ends, Laplacian
  ``edge=True`` ends) follow the published PyLops 1.x algorithm and are
  **parity unpinned** beyond adjoint dot-tests (no reference fixture holds
  them).
"""
