"""Iterative-algorithm driver (mirrors ``pycsou/core/solver.py``).

``iterate`` keeps the reference loop condition exactly
(``while ((iter <= max_iter) and (stopping_metric() > accuracy_threshold)) or (iter <= min_iter)``,
``solver.py:65-66``), returns ``(iterand, True, diagnostics)`` (``converged`` is always
``True``, ``solver.py:74``) and supports ``iterates(n)`` / ``reset``.  Subclasses that
own a fused device engine (``PrimalDualSplitting``) override ``iterate`` with a
hipGraph-replayed loop whose device-side stop flag implements the same condition.
"""

from abc import ABC, abstractmethod


def _snapshot(iterand):
    """Copy of the iterand dict (the reference deep-copies it every iteration, solver.py:72)."""
    if isinstance(iterand, dict):
        return {k: (v.clone() if hasattr(v, 'clone') else (v.copy() if hasattr(v, 'copy') else v))
                for k, v in iterand.items()}
    return iterand


class GenericIterativeAlgorithm(ABC):
    """``pycsou/core/solver.py:17-134``."""

    def __init__(self, objective_functional, init_iterand, max_iter=500, min_iter=10, accuracy_threshold=1e-3,
                 verbose=None):
        self.objective_functional = objective_functional
        self.max_iter = max_iter
        self.min_iter = min_iter
        self.accuracy_threshold = accuracy_threshold
        self.verbose = verbose
        self.diagnostics = None
        self.iter = 0
        self.iterand = None
        self.init_iterand = init_iterand
        self.converged = False

    def iterate(self):
        self.old_iterand = _snapshot(self.init_iterand)
        while ((self.iter <= self.max_iter) and (self.stopping_metric() > self.accuracy_threshold)) or (
                self.iter <= self.min_iter):
            self.iterand = self.update_iterand()
            self.update_diagnostics()
            if self.verbose is not None and self.iter % self.verbose == 0:
                self.print_diagnostics()
            self.old_iterand = _snapshot(self.iterand)
            self.iter += 1
        self.converged = True
        self.iterand = self.postprocess_iterand()
        return self.iterand, self.converged, self.diagnostics

    def postprocess_iterand(self):
        return self.iterand

    def reset(self):
        self.iter = 0
        self.iterand = None

    def iterates(self, n):
        self.reset()
        for _ in range(n):
            self.iterand = self.update_iterand()
            self.iter += 1
            yield self.iterand

    @abstractmethod
    def update_iterand(self):
        pass

    @abstractmethod
    def print_diagnostics(self):
        pass

    @abstractmethod
    def stopping_metric(self):
        pass

    @abstractmethod
    def update_diagnostics(self):
        pass
