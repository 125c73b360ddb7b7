"""Native scheduler policies (mirrors master/internal/rm/agentrm/*_test.go behaviours)."""
from determined_clone_amd.native import load

N = load()


def agent(aid, slots=8, used=None, pool="default"):
    a = N.Agent()
    a.id = aid
    a.num_slots = slots
    owners = [""] * slots
    for i, o in (used or {}).items():
        owners[i] = o
    a.slot_owner = owners
    a.slot_enabled = [True] * slots
    a.pool = pool
    return a


def req(aid, slots=1, prio=42, job=None, t=0.0, preemptible=True, weight=1.0):
    r = N.Request()
    r.alloc_id = aid
    r.job_id = job or aid
    r.slots = slots
    r.priority = prio
    r.submit_time = t
    r.preemptible = preemptible
    r.weight = weight
    return r


def run(aid, slots, prio=42, job=None, t=0.0, preemptible=True, weight=1.0):
    r = N.Running()
    r.alloc_id = aid
    r.job_id = job or aid
    r.slots = slots
    r.priority = prio
    r.start_time = t
    r.preemptible = preemptible
    r.weight = weight
    return r


def starts(d):
    return {a: [(p.agent_id, list(p.slots)) for p in ps] for a, ps in d.start}


def test_gang_placement_contiguous_on_one_agent():
    s = N.Scheduler("priority", "best", True)
    d = s.schedule([agent("a0", used={0: "x", 2: "y"})], [req("t1", slots=4)], [])
    got = starts(d)["t1"]
    assert got == [("a0", [3, 4, 5, 6])]


def test_best_fit_packs_worst_fit_spreads():
    agents = [agent("a0", used={i: "x" for i in range(6)}), agent("a1")]
    best = starts(N.Scheduler("priority", "best", True).schedule(agents, [req("t", 2)], []))
    worst = starts(N.Scheduler("priority", "worst", True).schedule(agents, [req("t", 2)], []))
    assert best["t"][0][0] == "a0"
    assert worst["t"][0][0] == "a1"


def test_multi_agent_dedicated_fit():
    agents = [agent("a0"), agent("a1"), agent("a2", used={0: "x"})]
    d = N.Scheduler("priority", "best", True).schedule(agents, [req("big", 16)], [])
    got = starts(d)["big"]
    assert sorted(a for a, _ in got) == ["a0", "a1"]
    assert all(len(s) == 8 for _, s in got)


def test_sixteen_single_slot_trials_fill_node_in_order():
    # ASHA with 16 concurrent 1-slot trials on one 8-GPU node: 8 start, 8 wait
    reqs = [req(f"t{i:02d}", 1, t=i) for i in range(16)]
    d = N.Scheduler("priority", "best", True).schedule([agent("n0")], reqs, [])
    st = starts(d)
    assert sorted(st) == [f"t{i:02d}" for i in range(8)]
    assert sorted(s[0][1][0] for s in st.values()) == list(range(8))


def test_priority_preemption():
    agents = [agent("a0", used={i: "low" for i in range(8)})]
    d = N.Scheduler("priority", "best", True).schedule(
        agents, [req("high", 4, prio=10)], [run("low", 8, prio=50)])
    assert list(d.preempt) == ["low"]
    assert "high" not in starts(d)  # starts once the victim releases its slots


def test_no_preemption_of_higher_or_nonpreemptible():
    agents = [agent("a0", used={i: "r" for i in range(8)})]
    s = N.Scheduler("priority", "best", True)
    assert list(s.schedule(agents, [req("p", 4, prio=50)], [run("r", 8, prio=10)]).preempt) == []
    assert list(s.schedule(agents, [req("p", 4, prio=10)],
                           [run("r", 8, prio=50, preemptible=False)]).preempt) == []


def test_strict_priority_without_preemption_blocks_lower():
    agents = [agent("a0", 4)]
    d = N.Scheduler("priority", "best", False).schedule(
        agents, [req("big", 8, prio=10), req("small", 1, prio=50)], [])
    assert starts(d) == {}


def test_round_robin_fifo():
    agents = [agent("a0", 4)]
    d = N.Scheduler("round_robin", "best", False).schedule(
        agents, [req("b", 3, t=2), req("a", 2, t=1), req("c", 2, t=3)], [])
    assert sorted(starts(d)) == ["a", "c"]


def test_fair_share_splits_by_weight():
    agents = [agent("a0", 8)]
    reqs = [req(f"j1-{i}", 1, job="j1", t=i) for i in range(8)] + \
           [req(f"j2-{i}", 1, job="j2", t=i, weight=3.0) for i in range(8)]
    d = N.Scheduler("fair_share", "best", True).schedule(agents, reqs, [])
    st = starts(d)
    n1 = sum(1 for k in st if k.startswith("j1"))
    n2 = sum(1 for k in st if k.startswith("j2"))
    assert (n1, n2) == (2, 6)


def test_fair_share_preempts_over_share_group():
    agents = [agent("a0", 8, used={i: f"j1-{i}" for i in range(8)})]
    running = [run(f"j1-{i}", 1, job="j1", t=i) for i in range(8)]
    d = N.Scheduler("fair_share", "best", True).schedule(agents, [req("j2-0", 4, job="j2")], running)
    assert len(d.preempt) == 4
    # oldest request first, as the reference's assignTasks (fair_share_test.go
    # TestFairShareMaxSlotsReleaseAllocatedTasks releases task1 and task2)
    assert set(d.preempt) == {f"j1-{i}" for i in range(4)}


def test_detect_kfd_on_fake_sysfs(tmp_path):
    node = tmp_path / "sys/class/kfd/kfd/topology/nodes"
    (node / "0").mkdir(parents=True)
    (node / "0/properties").write_text("simd_count 0\n")
    (node / "1/mem_banks/0").mkdir(parents=True)
    (node / "1/properties").write_text(
        "simd_count 1024\nsimd_per_cu 4\ngfx_target_version 90500\nunique_id 1234\nlocation_id 512\n"
        "drm_render_minor 128\nvendor_id 4098\ndevice_id 29857\n")
    (node / "1/mem_banks/0/properties").write_text("size_in_bytes 309220868096\n")
    gpus = N.detect_kfd_gpus(str(tmp_path))
    assert len(gpus) == 1
    g = gpus[0]
    assert g["gfx_target"] == "gfx950" and g["cu_count"] == "256" and g["index"] == "0"
