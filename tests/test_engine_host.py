"""Host logic of GpuBlupEngine that needs no GPU: the split cache (an IntraGCV call
with more folds than the cache holds must not evict its own earlier folds)."""
from collections import OrderedDict

import numpy as np

from tblup_amd.engine import GpuBlupEngine


class _FakeLib:
    def __init__(self):
        self.live = set()
        self.dropped = []

    def tblup_set_split(self, ctx, sid, *a):
        self.live.add(sid)
        return 0

    def tblup_drop_split(self, ctx, sid):
        assert sid in self.live
        self.live.remove(sid)
        self.dropped.append(sid)
        return 0


def _engine():
    eng = GpuBlupEngine.__new__(GpuBlupEngine)
    eng._lib = _FakeLib()
    eng._ctx = None
    eng._splits = OrderedDict()
    eng._next_split = 0
    eng._pending = None
    return eng


def _splits(n, seed):
    rng = np.random.default_rng(seed)
    return [(rng.permutation(100)[:60], rng.permutation(100)[:20]) for _ in range(n)]


def test_one_call_never_evicts_its_own_splits():
    eng = _engine()
    old = _splits(GpuBlupEngine.MAX_SPLITS, 0)
    eng.split_ids(old)
    folds = _splits(GpuBlupEngine.MAX_SPLITS + 5, 1)       # more folds than the cache holds
    ids = eng.split_ids(folds)
    assert len(set(ids)) == len(folds)
    assert set(ids) <= eng._lib.live                       # every fold of the call is registered
    assert len(eng._lib.dropped) == GpuBlupEngine.MAX_SPLITS   # the older call's splits went first
    # a later single registration shrinks the cache back to its bound
    eng.split_id(*_splits(1, 2)[0])
    assert len(eng._splits) <= len(folds) + 1
    assert eng._lib.live == {v[0] for v in eng._splits.values()}


def test_cached_split_ids_are_stable():
    eng = _engine()
    s = _splits(3, 3)
    a = eng.split_ids(s)
    b = eng.split_ids(s)
    assert a == b and not eng._lib.dropped
