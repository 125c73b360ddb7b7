"""The reference's fair-share and priority scheduler test vectors
(master/internal/rm/agentrm/{fair_share,priority}_test.go), ported case by case onto the native
scheduler (native/scheduler.cpp). priority_test.go's TestSortTasksByPriorityAndTimestamps checks an
internal sort helper and is covered through the queue-order cases instead.

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


# ------------------------------------------------------------------------------ priority.go
# master/internal/rm/agentrm/priority_test.go, on Scheduler("priority"). Multi-round cases follow
# its AllocateTasks / AddUnallocatedTasks / RemoveTask helpers: a started task takes the slots of
# the placement the scheduler returned and becomes a running allocation; removing it frees them.
# Tasks marked ``started`` begin on their agent with their slots (or zero-slot container) held.


@dataclass
class PAgent:
    id: str
    slots: int = 0
    max_zero: int = 0


@dataclass
class PTask:
    id: str
    slots: int
    priority: int
    job: Optional[str] = None
    started_on: Optional[PAgent] = None
    non_preemptible: bool = False


class PrioritySim:
    def __init__(self, agents, tasks, preemption):
        self.sched = N.Scheduler("priority", "best", preemption)
        self.agents = {}
        for a in agents:
            x = N.Agent()
            x.id, x.num_slots, x.max_zero_slot = a.id, a.slots, a.max_zero
            x.slot_owner, x.slot_enabled = [""] * a.slots, [True] * a.slots
            self.agents[a.id] = x
        self.pending, self.running, self.clock, self.positions = {}, {}, 0.0, {}
        for t in tasks:
            self.add(t)

    def _job(self, t):
        return t.job or t.id

    def add(self, t):
        self.clock += 1.0
        if t.started_on is not None:
            r = N.Running()
            r.alloc_id, r.job_id, r.slots, r.priority = t.id, self._job(t), t.slots, t.priority
            r.preemptible = not t.non_preemptible
            r.submit_time = r.job_submit_time = self.clock
            a = self.agents[t.started_on.id]
            if t.slots == 0:
                a.zero_slot_used += 1
            else:
                owners = list(a.slot_owner)
                free = [i for i, o in enumerate(owners) if not o][: t.slots]
                for i in free:
                    owners[i] = t.id
                a.slot_owner = owners
            r.agents = [a.id]
            self.running[t.id] = r
        else:
            r = N.Request()
            r.alloc_id, r.job_id, r.slots, r.priority = t.id, self._job(t), t.slots, t.priority
            r.preemptible = not t.non_preemptible
            r.submit_time = r.job_submit_time = self.clock
            self.pending[t.id] = r

    def schedule(self, positions=None):
        pend = list(self.pending.values())
        run = list(self.running.values())
        for x in pend + run:
            x.job_position = float((positions or {}).get(x.job_id, 0.0))
        d = self.sched.schedule(list(self.agents.values()), pend, run)
        return d

    def allocate(self, d):
        for alloc, places in d.start:
            req = self.pending.pop(alloc)
            r = N.Running()
            r.alloc_id, r.job_id, r.slots, r.priority = req.alloc_id, req.job_id, req.slots, req.priority
            r.preemptible, r.submit_time, r.job_submit_time = req.preemptible, req.submit_time, req.job_submit_time
            r.agents = [p.agent_id for p in places]
            for p in places:
                a = self.agents[p.agent_id]
                if not p.slots:
                    a.zero_slot_used += 1
                owners = list(a.slot_owner)
                for i in p.slots:
                    assert not owners[i], "slot handed out twice"
                    owners[i] = alloc
                a.slot_owner = owners
            self.running[alloc] = r

    def remove(self, alloc):
        r = self.running.pop(alloc)
        for aid in r.agents:
            a = self.agents[aid]
            if r.slots == 0:
                a.zero_slot_used -= 1
            a.slot_owner = ["" if o == alloc else o for o in a.slot_owner]


def started(d):
    return {alloc for alloc, _ in d.start}


LOW, MED, HIGH = 50, 45, 40


def _std_tasks(zero_slot_4_and_6=True):
    # task1..6 of PreemptionDisabled / AddTasks / AllSlotsAllocated / AllTasksFinished
    s4, s6 = (0, 0) if zero_slot_4_and_6 else (1, 1)
    return [PTask("task1", 4, LOW, "g1"), PTask("task2", 1, LOW, "g1"), PTask("task3", 1, HIGH, "g2"),
            PTask("task4", s4, HIGH, "g2"), PTask("task5", 4, HIGH, "g2"), PTask("task6", s6, LOW, "g1")]


def test_priority_max_zero_slot_container():
    sim = PrioritySim([PAgent("agent1", 4, 0)], [PTask("task1", 4, HIGH, "g2"), PTask("task6", 0, LOW, "g1")], True)
    assert started(sim.schedule()) == {"task1"}


def test_priority_preemption_disabled():
    sim = PrioritySim([PAgent("agent1", 4, 100), PAgent("agent2", 4, 100)], _std_tasks(), False)
    assert started(sim.schedule()) == {"task2", "task3", "task4", "task5", "task6"}
    # the scheduler works on copies: the caller's agent state is untouched
    assert all(not any(a.slot_owner) for a in sim.agents.values())


def test_priority_preemption_disabled_higher_priority_blocks_lower_priority():
    sim = PrioritySim([PAgent("agent1", 4), PAgent("agent2", 4)],
                      [PTask("task1", 4, LOW, "g1"), PTask("task2", 1, LOW, "g1"), PTask("task3", 12, HIGH, "g2")], False)
    assert started(sim.schedule()) == set()


def test_priority_preemption_disabled_add_tasks():
    sim = PrioritySim([PAgent("agent1", 4, 100), PAgent("agent2", 4, 100)], _std_tasks(), False)
    d = sim.schedule()
    assert started(d) == {"task2", "task3", "task4", "task5", "task6"}
    sim.allocate(d)
    for i in (7, 8, 9):
        sim.add(PTask(f"task{i}", 1, LOW, "g1"))
    assert started(sim.schedule()) == {"task7", "task8"}


def test_priority_preemption_disabled_all_slots_allocated():
    sim = PrioritySim([PAgent("agent1", 4), PAgent("agent2", 4)], _std_tasks(False), False)
    d = sim.schedule()
    assert started(d) == {"task2", "task3", "task4", "task5", "task6"}
    sim.allocate(d)
    sim.add(PTask("task7", 1, HIGH, "g2"))
    sim.add(PTask("task8", 1, HIGH, "g2"))
    assert started(sim.schedule()) == set()


def test_priority_preemption_disabled_lower_priority_must_wait():
    sim = PrioritySim([PAgent("agent1", 4)],
                      [PTask("task1", 1, LOW, "g1"), PTask("task2", 1, HIGH, "g2"), PTask("task3", 1, HIGH, "g2"),
                       PTask("task4", 1, HIGH, "g2"), PTask("task5", 2, HIGH, "g2")], False)
    d1 = sim.schedule()
    assert started(d1) == {"task2", "task3", "task4"}
    sim.allocate(d1)
    assert started(sim.schedule()) == set()
    for alloc in started(d1):
        sim.remove(alloc)
    assert started(sim.schedule()) == {"task1", "task5"}


def test_priority_preemption_disabled_task_finished():
    sim = PrioritySim([PAgent("agent1", 4, 100)], [PTask("task1", 4, HIGH, "g1")], False)
    d = sim.schedule()
    sim.allocate(d)
    sim.remove("task1")
    for t in (PTask("task7", 1, HIGH, "g1"), PTask("task8", 1, HIGH, "g1"), PTask("task9", 0, HIGH, "g1")):
        sim.add(t)
    assert started(sim.schedule()) == {"task7", "task8", "task9"}


def test_priority_preemption_disabled_all_tasks_finished():
    sim = PrioritySim([PAgent("agent1", 4), PAgent("agent2", 4)], _std_tasks(False), False)
    d = sim.schedule()
    assert started(d) == {"task2", "task3", "task4", "task5", "task6"}
    sim.allocate(d)
    sim.add(PTask("task7", 4, HIGH, "g2"))
    for alloc in started(d):
        sim.remove(alloc)
    assert started(sim.schedule()) == {"task1", "task7"}


def test_priority_preemption_disabled_zero_slot_task():
    sim = PrioritySim([PAgent("agent1", 4, 1)], [PTask("task1", 0, LOW, "g1"), PTask("task2", 0, LOW, "g1")], False)
    d = sim.schedule()
    assert started(d) == {"task1"}
    sim.allocate(d)
    sim.add(PTask("task3", 0, HIGH, "g2"))
    d = sim.schedule()
    assert started(d) == set() and set(d.preempt) == set()


def test_priority_preemption():
    a1, a2 = PAgent("agent1", 4), PAgent("agent2", 4)
    sim = PrioritySim([a1, a2], [
        PTask("low-priority task cannot be backfilled because preemption exists", 1, LOW, "g1"),
        PTask("medium-priority task should be preempted", 4, MED, "g2", started_on=a1),
        PTask("high-priority task should not be preempted", 4, HIGH, "g3", started_on=a2),
        PTask("high-priority task causes preemption but should not be scheduled", 4, HIGH, "g3"),
        PTask("high-priority oversized task triggers backfilling", 8, HIGH, "g3")], True)
    d = sim.schedule()
    assert started(d) == set()
    assert set(d.preempt) == {"medium-priority task should be preempted"}


def test_priority_backfilling():
    a1, a2 = PAgent("agent1", 4), PAgent("agent2", 4)
    sim = PrioritySim([a1, a2], [
        PTask("low-priority task should be preempted", 1, 55, "g1", started_on=a1),
        PTask("lower-priority task causes preemption but should not be scheduled", 1, 50, "g2"),
        PTask("medium-priority task should be backfilled", 1, 45, "g3"),
        PTask("high-priority task should not be preempted", 4, 40, "g4", started_on=a2),
        PTask("high-priority task should be scheduled", 2, 40, "g4"),
        PTask("high-priority oversized task triggers backfilling", 8, 40, "g4")], True)
    d = sim.schedule()
    assert started(d) == {"medium-priority task should be backfilled", "high-priority task should be scheduled"}
    assert set(d.preempt) == {"low-priority task should be preempted"}


def test_priority_preemption_zero_slot_task():
    a1, a2 = PAgent("agent1", 0, 1), PAgent("agent2", 0, 1)
    sim = PrioritySim([a1, a2], [
        PTask("low-priority task cannot be scheduled", 0, LOW, "g1"),
        PTask("medium-priority task should be preempted", 0, MED, "g2", started_on=a1),
        PTask("high-priority task should not be preempted", 0, HIGH, "g3", started_on=a2),
        PTask("high-priority task causes preemption but should not be scheduled", 0, HIGH, "g3")], True)
    d = sim.schedule()
    assert started(d) == set()
    assert set(d.preempt) == {"medium-priority task should be preempted"}


def test_priority_backfilling_zero_slot_task():
    a1, a2 = PAgent("agent1", 0, 4), PAgent("agent2", 0, 1)
    sim = PrioritySim([a1, a2], [
        PTask("low-priority task should be scheduled", 0, 55, "g1"),
        PTask("medium-priority task should not be preempted", 0, 50, "g2", started_on=a1),
        PTask("high-priority task should not be preempted", 0, 45, "g3", started_on=a2),
        PTask("high-priority task should be scheduled", 0, 45, "g3")], True)
    d = sim.schedule()
    assert started(d) == {"low-priority task should be scheduled", "high-priority task should be scheduled"}
    assert set(d.preempt) == set()


@pytest.mark.parametrize("positions", [{"1": 1, "2": 2, "3": 1.5}, {"1": 1, "2": 1, "3": 0.999}])
def test_priority_preempt_one_by_position(positions):
    a1, a2 = PAgent("agent1", 4), PAgent("agent2", 4)
    sim = PrioritySim([a1, a2], [PTask("1", 1, 42, "1", started_on=a1), PTask("2", 4, 42, "2", started_on=a2),
                                 PTask("3", 4, 42, "3")], True)
    d = sim.schedule(positions)
    assert started(d) == set() and set(d.preempt) == {"2"}


def test_priority_no_preemption_by_position():
    a1, a2 = PAgent("agent1", 4), PAgent("agent2", 4)
    sim = PrioritySim([a1, a2], [PTask("1", 1, 42, "1", started_on=a1), PTask("2", 4, 42, "2", started_on=a2),
                                 PTask("3", 8, 42, "3")], True)
    # job 3 sits between jobs 1 and 2: only job 2 is behind it, and freeing job 2 is not enough
    d = sim.schedule({"1": 1, "2": 2, "3": 1.5})
    assert started(d) == set() and set(d.preempt) == set()
