"""Multilevel hierarchy container (MLHierarchy.py:1-78): operators on the host (setup data).

Level 0 is the coarsest, numLevels-1 the finest. update(k) = I_up[k] maps level k to k+1,
downdate(k) = I_down[k] maps k+1 to k, matrix(k) = A[k] = I_down[k] (A[k+1] I_up[k]).
"""
from abc import ABC, abstractmethod


class MLHierarchy(ABC):
    def __init__(self, numLevels=2, normalize=True):
        self._numLevels = numLevels
        self._ops = [None] * numLevels
        self._updates = [None] * numLevels
        self._downdates = [None] * numLevels
        self._normalize = normalize

    @abstractmethod
    def makeProlongator(self, k):
        ...

    def numLevels(self):
        return self._numLevels

    def update(self, k):
        return self._updates[k]

    def downdate(self, k):
        return self._downdates[k]

    def matrix(self, k):
        return self._ops[k]

    def _setUpdate(self, k, I_up):
        self._updates[k] = I_up
        self._downdates[k] = makeRestrictionOp(I_up, self._normalize)
        self._ops[k] = self._downdates[k] * (self._ops[k + 1] * self._updates[k])

    def _setFineMatrix(self, A_fine):
        self._ops[self._numLevels - 1] = A_fine


def makeRestrictionOp(I_up, normalize=True):
    """I_down = I_up^T (MLHierarchy.py:304-322), sorted columns, duplicates summed.

    The reference's optional row normalisation never reaches the returned matrix (it rescales a
    lil row VIEW whose __itruediv__ rebinds the view's lists, :316-319); measured on DH-8 the
    reference returns I_up^T exactly, so ``normalize`` is accepted and has the same (no) effect.
    """
    R = I_up.transpose(copy=True).tocsr()
    R.sum_duplicates()
    return R
