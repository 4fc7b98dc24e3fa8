"""The brain's care of the collector's frozen generation:
frozen once after the first fleet-sized planning cycle; a later one, or an
idle tick at most every GC_IDLE_EVERY_S, thaws it, runs a full collection
(cyclic garbage of jobs that closed since) and freezes again."""
import gc

from foremast_amd.config import BrainConfig
from foremast_amd.engine.brain import Brain
from foremast_amd.engine.sources import SourceRouter
from foremast_amd.service.store import MemoryStore


class _Cyc:
    def __init__(self):
        self.me = self


def test_gc_freeze_is_maintained_not_repeated():
    b = Brain(MemoryStore(), BrainConfig(), sources=SourceRouter.synthetic_only())
    try:
        b.gc_maintenance(idle=True)                  # nothing frozen yet: no-op
        assert getattr(b, "gc_collections", 0) == 0 and getattr(b, "_gc_frozen_at", None) is None
        b.gc_maintenance(refreeze=True)              # the first big planning cycle
        assert gc.get_freeze_count() > 0 and getattr(b, "gc_collections", 0) == 0
        garbage = [_Cyc() for _ in range(100)]       # cycles created after the freeze ...
        del garbage
        b.gc_maintenance(idle=True)                  # ... an idle tick inside the interval: no collection
        assert getattr(b, "gc_collections", 0) == 0
        b._gc_frozen_at -= b.GC_IDLE_EVERY_S + 1     # interval passed
        b.gc_maintenance(idle=True)
        assert b.gc_collections == 1 and gc.get_freeze_count() > 0
        b.gc_maintenance(refreeze=True)              # a later big planning cycle: thaw, collect, freeze
        assert b.gc_collections == 2
    finally:
        gc.unfreeze()


def test_steady_cycles_after_a_planning_cycle_do_not_collect(monkeypatch):
    """Regression: a steady cycle that reuses the previous claim batch planned
    nothing, so it must not re-run the thaw + full collection (it did when
    the planner's job count carried over: ~0.3 s per cycle at 10k jobs)."""
    from foremast_amd.engine import brain as brain_mod
    from tests.test_fastpath_models import _brain, _submit
    monkeypatch.setattr(brain_mod, "GC_FREEZE_AFTER", 3)
    clock, store, client, b, _ = _brain(True, "holt_winters", {})
    calls = []
    real = b.gc_maintenance
    monkeypatch.setattr(b, "gc_maintenance", lambda **kw: (calls.append(kw), real(**kw)))
    try:
        _submit(client, "continuous")
        for _ in range(4):
            b.run_once()
            clock.t += 60.0
        assert b.fast.new_jobs == 0
        assert calls == [{"refreeze": True}]         # the planning cycle only
    finally:
        gc.unfreeze()


def test_steady_cycles_freeze_their_survivors_and_collect_periodically(monkeypatch):
    """Once frozen, each steady cycle ends with gc.freeze() (O(1)): the
    automatic collections only walk the cycle's young objects; a thaw + full
    collection runs when GC_FULL_EVERY_S has passed since the last freeze."""
    from foremast_amd.engine import brain as brain_mod
    from tests.test_fastpath_models import _brain, _submit
    monkeypatch.setattr(brain_mod, "GC_FREEZE_AFTER", 3)
    clock, store, client, b, _ = _brain(True, "holt_winters", {})
    try:
        _submit(client, "continuous")
        b.run_once()                                   # planning cycle: the first freeze
        clock.t += 60.0
        assert b._gc_frozen_at is not None and getattr(b, "gc_collections", 0) == 0
        kept = _Cyc()                                  # survives the cycle: frozen at its end
        b.run_once()                                   # a steady cycle: its survivors frozen
        clock.t += 60.0
        assert getattr(b, "gc_collections", 0) == 0
        assert not any(o is kept for o in gc.get_objects())   # (get_objects skips the frozen generation)
        b._gc_frozen_at -= b.GC_FULL_EVERY_S + 1       # the full-collection interval passed
        b.run_once()
        assert b.gc_collections == 1 and gc.get_freeze_count() > 0
    finally:
        gc.unfreeze()
