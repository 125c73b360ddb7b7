"""The reference's fair-share scheduler test vectors (master/internal/rm/agentrm/fair_share_test.go),
ported case by case onto the native scheduler (native/scheduler.cpp ``Scheduler("fair_share")``).

Harness semantics follow the reference's setupSchedulerStates (scheduler_test.go:451-544):
* tasks are submitted in list order (each gets a later submission time); a task without a group
  forms its own job; groups / implicit jobs have weight 0 and no max_slots unless given;
* an ``allocated`` task is a running allocation whose container has not started: it does not
  occupy device slots in the agent state (the reference's ContainerStarted=false "proxy to
  oversubscribe agents"), so pending tasks may still fit on its agent;
* assertions compare the SETS of started and released allocations, like assertEqualToAllocate /
  assertEqualToRelease.

One deliberate difference: TestFairShareBlocklistMultiple lists two 8-slot tasks that both fit on
the same two free agents and expects BOTH in toAllocate (its comment: "allocateResources should
handle this case and only let us schedule one of these at a time"). Our scheduler returns concrete
slot placements that the master applies directly, so it places the first and not the second within
one call -- the outcome the reference reaches after its allocation step.
"""
from dataclasses import dataclass, field
from typing import List, Optional

import pytest

from determined_clone_amd.native import load

N = load()


@dataclass
class MAgent:
    id: str
    slots: int


@dataclass
class MGroup:
    id: str
    max_slots: Optional[int] = None
    weight: float = 0.0


@dataclass
class MTask:
    id: str
    slots: int
    group: Optional[MGroup] = None
    allocated: Optional[MAgent] = None
    non_preemptible: bool = False
    blocked: List[str] = field(default_factory=list)


def run_fair_share(agents, tasks):
    na = []
    for a in agents:
        x = N.Agent()
        x.id, x.num_slots = a.id, a.slots
        x.slot_owner = [""] * a.slots
        x.slot_enabled = [True] * a.slots
        na.append(x)
    pend, run = [], []
    for i, t in enumerate(tasks):
        g = t.group
        job = g.id if g else t.id
        weight = g.weight if g else 0.0
        max_slots = g.max_slots if g and g.max_slots is not None else -1
        if t.allocated is not None:
            r = N.Running()
            r.alloc_id, r.job_id, r.slots = t.id, job, t.slots
            r.weight, r.max_slots, r.preemptible = weight, max_slots, not t.non_preemptible
            r.submit_time = r.job_submit_time = float(i)
            run.append(r)
        else:
            r = N.Request()
            r.alloc_id, r.job_id, r.slots = t.id, job, t.slots
            r.weight, r.max_slots, r.preemptible = weight, max_slots, not t.non_preemptible
            r.submit_time = r.job_submit_time = float(i)
            r.blocked_agents = list(t.blocked)
            pend.append(r)
    d = N.Scheduler("fair_share", "best", True).schedule(na, pend, run)
    started = {alloc for alloc, _ in d.start}
    return started, set(d.preempt)


def ids(*tasks):
    return {t.id for t in tasks}


def test_fair_share_max_slots():
    agents = [MAgent("agent", 4)]
    g1, g2 = MGroup("group1", max_slots=1, weight=1), MGroup("group2")
    t = [MTask(f"task{i + 1}", 1, g1 if i < 4 else g2) for i in range(8)]
    assert run_fair_share(agents, t) == (ids(t[0], t[4], t[5], t[6]), set())


def test_fair_share_weights():
    agents = [MAgent("agent", 8)]
    g1, g2 = MGroup("group1", 100, 10), MGroup("group2", 100, 30)
    t = [MTask(f"task{i + 1}", 1, g1 if i < 3 else g2) for i in range(10)]
    assert run_fair_share(agents, t) == (ids(t[0], t[1], t[3], t[4], t[5], t[6], t[7], t[8]), set())


def test_fair_share_multi_slot():
    agents = [MAgent("agent1", 4), MAgent("agent2", 4)]
    g1, g2 = MGroup("group1"), MGroup("group2")
    t = [MTask("task1", 4, g1), MTask("task2", 4, g2)]
    assert run_fair_share(agents, t) == (ids(*t), set())


def test_fair_share_max_slots_release_allocated_tasks():
    a = MAgent("agent", 4)
    g1 = MGroup("group1", 2, 1)
    t = [MTask(f"task{i + 1}", 1, g1, allocated=a) for i in range(4)]
    assert run_fair_share([a], t) == (set(), ids(t[0], t[1]))


def test_fair_share_unscheduled():
    a1, a2 = MAgent("agent1", 2), MAgent("agent2", 2)
    g1 = MGroup("group1", 2, 1)
    t = [MTask("task1", 2, g1), MTask("task2", 1, g1, allocated=a1), MTask("task3", 1, g1, allocated=a2)]
    # the reference's allocated tasks do not occupy device slots (container not started), so
    # here task1 could fit -- but its group is already at max_slots with the two allocated ones
    assert run_fair_share([a1, a2], t) == (set(), set())


def test_fair_share_multi_slot_deadlock():
    agents = [MAgent("agent", 2)]
    g1, g2 = MGroup("group1"), MGroup("group2")
    t = [MTask("task1", 2, g1), MTask("task2", 2, g2)]
    assert run_fair_share(agents, t) == (ids(t[0]), set())


def test_fair_share_big_task():
    agents = [MAgent("agent", 4)]
    g1, g2 = MGroup("group1"), MGroup("group2")
    t = [MTask("task1", 5, g1), MTask("task2", 4, g2)]
    assert run_fair_share(agents, t) == (ids(t[1]), set())


def test_fair_share_active_tasks():
    a1, a2 = MAgent("agent1", 4), MAgent("agent2", 3)
    g = [MGroup(f"group{i + 1}") for i in range(4)]
    t = [MTask("task1", 3, g[0]), MTask("task2", 1, g[1]), MTask("task3", 1, g[1], allocated=a2),
         MTask("task4", 4, g[2]), MTask("task5", 1, g[3])]
    assert run_fair_share([a1, a2], t) == (ids(t[0], t[1], t[4]), set())


def test_fair_share_nil_group():
    a = MAgent("agent", 4)
    t = [MTask("task1", 4, allocated=a), MTask("task2", 1, allocated=a)]
    assert run_fair_share([a], t) == (set(), ids(t[0]))


def test_fair_share_preemptible():
    a = MAgent("agent", 1)
    t = [MTask("task1", 1, allocated=a), MTask("task2", 1, allocated=a)]
    assert run_fair_share([a], t) == (set(), ids(t[1]))


@pytest.mark.parametrize("first_non_preemptible", [False, True])
def test_fair_share_honors_non_preemptible_in_a_group(first_non_preemptible):
    a = MAgent("agent", 1)
    g1 = MGroup("group1", 2, 1)
    t = [MTask("task1", 1, g1, allocated=a, non_preemptible=first_non_preemptible),
         MTask("task2", 1, g1, allocated=a, non_preemptible=not first_non_preemptible)]
    released = t[1] if first_non_preemptible else t[0]
    assert run_fair_share([a], t) == (set(), ids(released))


@pytest.mark.parametrize("first_non_preemptible", [False, True])
def test_fair_share_honors_non_preemptible_nil_group(first_non_preemptible):
    a = MAgent("agent", 1)
    t = [MTask("task1", 1, allocated=a, non_preemptible=first_non_preemptible),
         MTask("task2", 1, allocated=a, non_preemptible=not first_non_preemptible)]
    released = t[1] if first_non_preemptible else t[0]
    assert run_fair_share([a], t) == (set(), ids(released))


def test_fair_share_blocklist():
    agents = [MAgent("agent", 1)]
    g0, g1 = MGroup("group0"), MGroup("group1")
    t = [MTask("task0.1", 1, g0, blocked=["agent"]), MTask("task1.1", 1, g1)]
    assert run_fair_share(agents, t) == (ids(t[1]), set())


def test_fair_share_blocklist_multiple():
    agents = [MAgent(f"agent{i}", 4) for i in range(4)]
    g0, g1 = MGroup("group0"), MGroup("group1")
    t = [MTask("task0.1", 8, g0, blocked=["agent2", "agent3"]),
         MTask("task1.1", 8, g1, blocked=["agent2", "agent3"])]
    # reference: both listed, its allocation step admits one (see the module docstring)
    assert run_fair_share(agents, t) == (ids(t[0]), set())


def test_fair_share_blocklist_preemptible():
    a0, a1 = MAgent("agent0", 1), MAgent("agent1", 1)
    t = [MTask("task0.1", 1, blocked=["agent0", "agent1"]), MTask("task1.1", 1, allocated=a0),
         MTask("task2.1", 1, blocked=["agent0"]), MTask("task3.1", 1, allocated=a1)]
    assert run_fair_share([a0, a1], t) == (ids(t[2]), ids(t[3]))


def test_fair_share_blocklist_dont_preempt():
    a0 = MAgent("agent0", 1)
    t = [MTask(f"task{i}.1", 1, blocked=["agent0"]) for i in range(3)] + [MTask("task3.1", 1, allocated=a0)]
    assert run_fair_share([a0], t) == (set(), set())


def test_fair_share_blocklist_equal():
    a0 = MAgent("agent0", 1)
    t = [MTask("task0.1", 1, blocked=["agent0"])] + [MTask(f"task{i}.1", 1, allocated=a0) for i in (1, 2, 3)]
    assert run_fair_share([a0], t) == (set(), ids(t[2], t[3]))


def test_fair_share_terminates_when_non_preemptible_exceed_max_slots():
    """Held non-preemptible slots above a (lowered) max_slots: the offer loop must still end
    (a negative offer used to spin -- found by the UBSan build, tests/test_native_sanitizers.py)."""
    a = MAgent("agent", 4)
    g1 = MGroup("group1", max_slots=1, weight=1)
    t = [MTask("task1", 1, g1, allocated=a, non_preemptible=True),
         MTask("task2", 1, g1, allocated=a, non_preemptible=True), MTask("task3", 1, g1)]
    assert run_fair_share([a], t) == (set(), set())
