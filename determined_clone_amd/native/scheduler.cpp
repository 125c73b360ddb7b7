// Native resource-manager scheduler: priority (with preemption/backfill), fair-share and
// round-robin policies, best/worst-fit slot placement and gang placement of multi-slot tasks.
//
// Reference behaviour: master/internal/rm/agentrm/{priority,fair_share,round_robin,fitting,
// fitting_methods}.go (Go). Re-designed for an MI355X node pool: an "agent" is one host with N
// GPU slots (8 x MI355X on xGMI); a task asking for <= N slots is always packed onto ONE agent so
// its ranks talk over xGMI, never over the host network; a task asking for more takes whole,
// fully idle agents (dedicated multi-agent fit). The scheduler is a pure function of the snapshot
// it is given (agents, pending requests, running allocations) -> decisions, so the master can
// call it from any thread and tests can drive it directly.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <functional>
#include <map>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace dca_native {

struct Agent {
  std::string id;
  int num_slots = 0;
  std::vector<std::string> slot_owner;  // "" = free, else allocation id
  std::vector<bool> slot_enabled;
  bool enabled = true;
  std::string pool;
  std::string label;
  int max_zero_slot = 100;
  int zero_slot_used = 0;

  int empty_slots() const {
    int n = 0;
    for (size_t i = 0; i < slot_owner.size(); ++i)
      if (slot_owner[i].empty() && slot_enabled[i]) ++n;
    return n;
  }
  int used_slots() const {
    int n = 0;
    for (auto& o : slot_owner)
      if (!o.empty()) ++n;
    return n;
  }
  int usable_slots() const {
    int n = 0;
    for (bool e : slot_enabled) n += e ? 1 : 0;
    return n;
  }
};

struct Request {
  std::string alloc_id;
  std::string job_id;
  int slots = 1;
  int priority = 42;  // smaller = more important (Determined convention)
  double weight = 1.0;
  double submit_time = 0.0;
  double job_position = 0;  // the job's queue position (UpdateJobQueue); smaller runs first
  bool preemptible = true;
  std::string pool;
  std::string label;
  std::vector<std::string> blocked_agents;
  int max_slots = -1;            // the job's resources.max_slots (fair share), -1 = unlimited
  double job_submit_time = 0.0;  // when the job (experiment / command) was submitted
};

struct Running {
  std::string alloc_id;
  std::string job_id;
  int slots = 0;
  int priority = 42;
  double weight = 1.0;
  double start_time = 0.0;
  bool preemptible = true;
  int max_slots = -1;
  double submit_time = 0.0;      // request submission (task-list order with the pending ones)
  double job_submit_time = 0.0;
  double job_position = 0;
  std::vector<std::string> agents;  // where it runs (zero-slot allocations hold no slot ids)
};

struct Placement {
  std::string agent_id;
  std::vector<int> slots;
};

struct Decision {
  std::vector<std::pair<std::string, std::vector<Placement>>> start;
  std::vector<std::string> preempt;
};

// ------------------------------------------------------------------ fitting
static uint64_t fnv1a(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) {
    h ^= c;
    h *= 1099511628211ull;
  }
  return h;
}

static double fit_score(const std::string& method, const Request& r, const Agent& a) {
  const int empty = a.empty_slots();
  if (method == "worst") {
    if (a.used_slots() != 0 || r.slots != 0) return static_cast<double>(empty) / std::max(1, a.usable_slots());
    return a.max_zero_slot ? static_cast<double>(a.max_zero_slot - a.zero_slot_used) / a.max_zero_slot : 0.0;
  }
  // best fit: most utilised agent with the fewest free slots
  if (a.used_slots() != 0 || r.slots != 0) return 1.0 / (1.0 + empty);
  return a.max_zero_slot ? 1.0 / (1.0 + (a.max_zero_slot - a.zero_slot_used)) : 0.0;
}

static bool agent_ok(const Request& r, const Agent& a) {
  if (!a.enabled) return false;
  if (!r.pool.empty() && a.pool != r.pool) return false;
  if (!r.label.empty() && a.label != r.label) return false;
  if (std::find(r.blocked_agents.begin(), r.blocked_agents.end(), a.id) != r.blocked_agents.end())
    return false;
  return true;
}

// Picks concrete slot indices on an agent; prefers a contiguous run so multi-GPU ranks share the
// same xGMI hive neighbourhood (contiguous device ids).
static std::vector<int> pick_slots(const Agent& a, int n) {
  std::vector<int> free;
  for (size_t i = 0; i < a.slot_owner.size(); ++i)
    if (a.slot_owner[i].empty() && a.slot_enabled[i]) free.push_back(static_cast<int>(i));
  if (static_cast<int>(free.size()) < n) return {};
  for (size_t s = 0; s + n <= free.size(); ++s)
    if (free[s + n - 1] - free[s] == n - 1) return std::vector<int>(free.begin() + s, free.begin() + s + n);
  return std::vector<int>(free.begin(), free.begin() + n);
}

// Returns placements (empty if it does not fit).
static std::vector<Placement> find_fit(const Request& r, const std::vector<Agent>& agents,
                                       const std::string& method) {
  if (r.slots == 0) {
    const Agent* best = nullptr;
    double bs = -1;
    for (auto& a : agents) {
      if (!agent_ok(r, a) || a.zero_slot_used >= a.max_zero_slot) continue;
      double s = fit_score(method, r, a);
      if (s > bs) { bs = s; best = &a; }
    }
    if (!best) return {};
    return {Placement{best->id, {}}};
  }
  // single-agent fit
  const Agent* best = nullptr;
  double bscore = -1;
  uint64_t bdist = 0;
  const uint64_t h = fnv1a(r.alloc_id);
  for (auto& a : agents) {
    if (!agent_ok(r, a) || a.empty_slots() < r.slots) continue;
    const double s = fit_score(method, r, a);
    const uint64_t d = fnv1a(a.id) ^ h;
    if (s > bscore + 1e-12 || (std::fabs(s - bscore) <= 1e-12 && d < bdist)) {
      best = &a;
      bscore = s;
      bdist = d;
    }
  }
  if (best) return {Placement{best->id, pick_slots(*best, r.slots)}};
  // dedicated multi-agent fit: whole idle agents of equal size
  std::vector<const Agent*> idle;
  for (auto& a : agents)
    if (agent_ok(r, a) && a.used_slots() == 0 && a.usable_slots() > 0) idle.push_back(&a);
  if (idle.empty()) return {};
  std::sort(idle.begin(), idle.end(), [](const Agent* x, const Agent* y) {
    return x->usable_slots() != y->usable_slots() ? x->usable_slots() > y->usable_slots() : x->id < y->id;
  });
  const int per = idle[0]->usable_slots();
  if (per == 0 || r.slots % per != 0) return {};
  const int need = r.slots / per;
  std::vector<Placement> out;
  for (auto* a : idle) {
    if (a->usable_slots() != per) continue;
    out.push_back(Placement{a->id, pick_slots(*a, per)});
    if (static_cast<int>(out.size()) == need) return out;
  }
  return {};
}

static void apply(std::vector<Agent>& agents, const std::string& alloc,
                  const std::vector<Placement>& ps) {
  for (auto& p : ps)
    for (auto& a : agents)
      if (a.id == p.agent_id) {
        if (p.slots.empty()) a.zero_slot_used++;
        for (int s : p.slots) a.slot_owner[s] = alloc;
      }
}

static void release(std::vector<Agent>& agents, const std::string& alloc, int zero_slots) {
  for (auto& a : agents) {
    for (auto& o : a.slot_owner)
      if (o == alloc) o.clear();
  }
  (void)zero_slots;
}

// Frees what running allocation ``r`` holds: its slots, or its zero-slot container count.
static void release_running(std::vector<Agent>& agents, const Running& r) {
  if (r.slots == 0) {
    for (auto& id : r.agents)
      for (auto& a : agents)
        if (a.id == id && a.zero_slot_used > 0) a.zero_slot_used--;
    return;
  }
  release(agents, r.alloc_id, 0);
}

// ------------------------------------------------------------------ policies
class Scheduler {
 public:
  Scheduler(std::string policy, std::string fit, bool preemption)
      : policy_(std::move(policy)), fit_(std::move(fit)), preemption_(preemption) {}

  Decision schedule(std::vector<Agent> agents, std::vector<Request> pending,
                    std::vector<Running> running) {
    if (policy_ == "fair_share") return fair_share(agents, pending, running);
    if (policy_ == "round_robin") return round_robin(agents, pending);
    return priority(agents, pending, running);
  }

 private:
  std::string policy_, fit_;
  bool preemption_;

  static bool req_order(const Request& a, const Request& b) {
    if (a.priority != b.priority) return a.priority < b.priority;
    if (a.job_position != b.job_position) return a.job_position < b.job_position;
    if (a.job_submit_time != b.job_submit_time) return a.job_submit_time < b.job_submit_time;
    if (a.submit_time != b.submit_time) return a.submit_time < b.submit_time;
    return a.alloc_id < b.alloc_id;
  }

  Decision round_robin(std::vector<Agent>& agents, std::vector<Request>& pending) {
    Decision d;
    std::sort(pending.begin(), pending.end(), [](const Request& a, const Request& b) {
      return a.submit_time != b.submit_time ? a.submit_time < b.submit_time : a.alloc_id < b.alloc_id;
    });
    for (auto& r : pending) {
      auto ps = find_fit(r, agents, fit_);
      if (ps.empty()) continue;
      apply(agents, r.alloc_id, ps);
      d.start.emplace_back(r.alloc_id, ps);
    }
    return d;
  }

  // Priority scheduling with preemption and backfilling, after the reference's priority.go
  // (prioritySchedulerWithFilter / trySchedulingTaskViaPreemption). Zero-slot and slot tasks are
  // scheduled independently. Per priority level (smallest number first), pending tasks are fitted
  // in queue order (position, job submission, request submission) onto a working copy of the
  // agents -- a fitted task holds its slots in that copy whether or not it is started -- and:
  //  * started only while nothing has been chosen for preemption; once some higher-priority task
  //    failed to fit, lower levels are "backfilling" and start only preemptible tasks (and only
  //    with preemption on);
  //  * a task that does not fit first checks whether the preemptions already chosen make room,
  //    else preempts running allocations from the lowest priority (99) up to its own level, newest
  //    in queue order first -- at its own level only jobs queued behind it -- until it fits; the
  //    victims are released only if it then fits.
  Decision priority(std::vector<Agent>& agents, std::vector<Request>& pending,
                    std::vector<Running>& running) {
    Decision d;
    std::sort(pending.begin(), pending.end(), req_order);
    std::vector<Running*> runs;
    for (auto& r : running) runs.push_back(&r);
    std::sort(runs.begin(), runs.end(), [](const Running* a, const Running* b) {
      if (a->priority != b->priority) return a->priority < b->priority;
      if (a->job_position != b->job_position) return a->job_position < b->job_position;
      if (a->job_submit_time != b->job_submit_time) return a->job_submit_time < b->job_submit_time;
      if (a->submit_time != b->submit_time) return a->submit_time < b->submit_time;
      return a->alloc_id < b->alloc_id;
    });
    constexpr int kMaxPriority = 99;
    for (int zero = 0; zero < 2; ++zero) {
      const bool want_zero = zero == 1;
      std::map<int, std::vector<Request*>> pend_by_prio;
      std::map<int, std::vector<Running*>> run_by_prio;
      for (auto& r : pending)
        if ((r.slots == 0) == want_zero) pend_by_prio[r.priority].push_back(&r);
      for (auto* r : runs)
        if ((r->slots == 0) == want_zero) run_by_prio[r->priority].push_back(r);
      std::vector<Agent> local = agents;
      bool backfilling = false;
      std::vector<std::string> to_release;
      auto released = [&](const std::string& id) {
        return std::find(to_release.begin(), to_release.end(), id) != to_release.end();
      };
      for (auto& kv : pend_by_prio) {
        const int prio = kv.first;
        std::vector<std::pair<Request*, std::vector<Placement>>> ok;
        std::vector<Request*> failed;
        for (Request* r : kv.second) {
          auto ps = find_fit(*r, local, fit_);
          if (ps.empty()) {
            failed.push_back(r);
            continue;
          }
          apply(local, r->alloc_id, ps);
          ok.emplace_back(r, ps);
        }
        if (to_release.empty()) {
          for (auto& rp : ok) {
            if (backfilling && !(preemption_ && rp.first->preemptible)) continue;
            apply(agents, rp.first->alloc_id, rp.second);
            d.start.emplace_back(rp.first->alloc_id, rp.second);
          }
        }
        if (!failed.empty()) backfilling = true;
        if (!preemption_) continue;
        for (Request* r : failed) {
          auto ps = find_fit(*r, local, fit_);
          if (!ps.empty()) {  // room once the already chosen preemptions complete
            apply(local, r->alloc_id, ps);
            continue;
          }
          std::vector<Agent> trial = local;
          std::vector<std::string> victims;
          bool placed = false;
          for (int p = kMaxPriority; p >= prio && !placed; --p) {
            auto it = run_by_prio.find(p);
            if (it == run_by_prio.end()) continue;
            auto& cands = it->second;
            for (int i = static_cast<int>(cands.size()) - 1; i >= 0; --i) {
              Running* c = cands[i];
              if (p == prio && r->job_position >= c->job_position) break;
              if (!c->preemptible || released(c->alloc_id)) continue;
              release_running(trial, *c);
              victims.push_back(c->alloc_id);
              auto fit = find_fit(*r, trial, fit_);
              if (!fit.empty()) {
                apply(trial, r->alloc_id, fit);
                placed = true;
                break;
              }
            }
          }
          if (placed) {
            local = std::move(trial);
            for (auto& v : victims) to_release.push_back(v);
          }
        }
      }
      for (auto& v : to_release) d.preempt.push_back(v);
    }
    return d;
  }

  // Max-min fair share over jobs ("groups"), following the reference's fair_share.go:
  //  1. every request (pending and running, in submission order) joins its job's group; pending
  //     ones that could not be placed even after preemption, and ones larger than the whole pool,
  //     are left out (they would waste offered slots); a group's demand is capped at max_slots;
  //  2. slots already held by non-preemptible allocations are offered first (pre-offers);
  //  3. progressive filling: groups in order of increasing demand (then age) each get
  //     max(1, capacity * weight / total_weight) per round until demands are met or the pool is
  //     empty; when it is empty and some group cannot start even its smallest task with what it
  //     was offered, the newest such group is disabled and its offer returned (multi-slot
  //     deadlock breaking);
  //  4. groups holding more than their offer release preemptible allocations (oldest request
  //     first) -- unless preemption is off; groups under it start pending tasks that fit.
  // Placements are applied as they are made, so one call never hands the same slots to two
  // tasks (the reference lists both and lets a later allocation step reject the second).
  Decision fair_share(std::vector<Agent>& agents, std::vector<Request>& pending,
                      std::vector<Running>& running) {
    Decision d;
    for (auto& r : pending) {  // zero-slot tasks need no offer, only room on an agent
      if (r.slots != 0) continue;
      auto ps = find_fit(r, agents, fit_);
      if (ps.empty()) continue;
      apply(agents, r.alloc_id, ps);
      d.start.emplace_back(r.alloc_id, ps);
    }
    int capacity = 0;
    for (auto& a : agents) capacity += a.usable_slots();

    struct Task {
      double t;
      size_t idx;
      Request* req;   // pending
      Running* run;   // allocated
      int slots() const { return req ? req->slots : run->slots; }
      bool preemptible() const { return req ? req->preemptible : run->preemptible; }
    };
    std::vector<Task> tasks;
    for (size_t i = 0; i < running.size(); ++i)
      tasks.push_back({running[i].submit_time, i, nullptr, &running[i]});
    for (size_t i = 0; i < pending.size(); ++i)
      tasks.push_back({pending[i].submit_time, running.size() + i, &pending[i], nullptr});
    std::stable_sort(tasks.begin(), tasks.end(), [](const Task& x, const Task& y) {
      return x.t != y.t ? x.t < y.t : x.idx < y.idx;
    });

    struct Group {
      std::string job;
      double weight = 1.0, registered = 0.0;
      int max_slots = -1, order = 0;
      bool disabled = false;
      int demand = 0, active = 0, presubscribed = 0, offered = 0;
      std::vector<Task> pend, alloc;
    };
    // A pending task counts toward its group's demand if it could be placed once the preemptible
    // allocations were released. (The reference checks the slots free right now, so on a full
    // pool a newly submitted job never receives a share and nothing is ever preempted for it;
    // its vectors, whose allocated tasks hold no device slots, behave the same under both rules.)
    std::vector<Agent> reclaimable = agents;
    if (preemption_)
      for (auto& run : running)
        if (run.preemptible) release(reclaimable, run.alloc_id, 0);
    std::vector<Group> groups;
    std::map<std::string, size_t> index;
    for (auto& t : tasks) {
      const int n = t.slots();
      if (n == 0 || n > capacity) continue;
      if (t.req && find_fit(*t.req, reclaimable, fit_).empty()) continue;
      const std::string& job = t.req ? t.req->job_id : t.run->job_id;
      auto it = index.find(job);
      if (it == index.end()) {
        Group g;
        g.job = job;
        g.weight = t.req ? t.req->weight : t.run->weight;
        g.max_slots = t.req ? t.req->max_slots : t.run->max_slots;
        g.registered = t.req ? t.req->job_submit_time : t.run->job_submit_time;
        g.order = static_cast<int>(groups.size());
        it = index.emplace(job, groups.size()).first;
        groups.push_back(std::move(g));
      }
      Group& g = groups[it->second];
      g.demand += n;
      if (t.req) {
        g.pend.push_back(t);
      } else {
        if (!t.preemptible()) g.presubscribed += n;
        g.active += n;
        g.alloc.push_back(t);
      }
    }
    for (auto& g : groups)
      if (g.max_slots >= 0) g.demand = std::min(g.demand, g.max_slots);

    // ---- slot offers
    std::map<int, int> preoffers;  // group order -> slots still pre-offered
    for (auto& g : groups) {
      if (g.presubscribed == 0) continue;
      g.offered = g.presubscribed;
      preoffers[g.order] = g.presubscribed;
      capacity -= g.presubscribed;
    }
    std::stable_sort(groups.begin(), groups.end(), [](const Group& x, const Group& y) {
      if (x.demand != y.demand) return x.demand < y.demand;
      return x.registered < y.registered;
    });
    std::vector<size_t> newest_first(groups.size());
    for (size_t i = 0; i < groups.size(); ++i) newest_first[i] = i;
    std::stable_sort(newest_first.begin(), newest_first.end(), [&](size_t x, size_t y) {
      if (groups[x].registered != groups[y].registered) return groups[x].registered > groups[y].registered;
      return groups[x].order > groups[y].order;
    });
    auto total_weight = [&]() {
      double w = 0;
      for (auto& g : groups)
        if (!g.disabled && g.offered < g.demand) w += g.weight;
      return w;
    };
    double tw = total_weight();
    // Rounds until every group is satisfied or disabled, or a round changes nothing. Offers are
    // clamped at zero: a group can hold more non-preemptible slots than its (max_slots-capped)
    // demand and the pool can be oversubscribed, and a negative offer would never terminate.
    for (;;) {
      bool open = false, progress = false;
      const int start_capacity = capacity;
      for (auto& g : groups) {
        if (g.disabled || g.offered >= g.demand) continue;
        open = true;
        // max(1, floor(share)); a pool of zero-weight groups fills one slot per group per round
        const int fair = tw > 0 ? std::max(1, static_cast<int>(start_capacity * g.weight / tw)) : 1;
        int offer = std::max(0, std::min({fair, capacity, g.demand - g.offered}));
        int& pre = preoffers[g.order];
        const int pre_before = pre;
        // the reference's accountForPreoffers, arithmetic kept as is
        if (pre > 0) {
          if (pre == offer) pre = offer = 0;
          if (pre > offer) { pre -= offer; offer = 0; }
          if (pre < offer) pre = 0;
        }
        progress = progress || offer > 0 || pre != pre_before;
        g.offered += offer;
        capacity -= offer;
        if (g.offered >= g.demand) tw = total_weight();
      }
      if (!open) break;
      if (capacity <= 0) {
        // multi-slot deadlock: the newest group whose offer cannot start even its smallest
        // pending task gives its offer back
        bool adjusted = false;
        for (size_t i : newest_first) {
          Group& g = groups[i];
          int smallest = -1;
          for (auto& t : g.pend) smallest = smallest < 0 ? t.slots() : std::min(smallest, t.slots());
          if (!g.disabled && g.offered < g.demand && smallest > g.offered) {
            capacity += g.offered;
            g.offered = 0;
            g.disabled = true;
            adjusted = true;
            tw = total_weight();
            break;
          }
        }
        if (!adjusted) break;
      } else if (!progress) {
        break;
      }
    }

    // ---- decisions
    for (auto& g : groups) {
      if (g.active > g.offered) {
        if (!preemption_) continue;
        for (auto& t : g.alloc) {
          if (!t.preemptible()) continue;
          d.preempt.push_back(t.run->alloc_id);
          g.active -= t.slots();
          if (g.active <= g.offered) break;
        }
      } else if (g.active < g.offered) {
        int room = g.offered - g.active;
        for (auto& t : g.pend) {
          if (t.slots() > room) continue;
          auto ps = find_fit(*t.req, agents, fit_);
          if (ps.empty()) continue;
          apply(agents, t.req->alloc_id, ps);
          d.start.emplace_back(t.req->alloc_id, ps);
          room -= t.slots();
        }
      }
    }
    return d;
  }
};

}  // namespace dca_native

// ------------------------------------------------------------------ device detection
#include <dirent.h>
#include <fstream>
#include <sstream>

namespace dca_native {

// Enumerate AMD GPUs from the KFD topology in sysfs (what the ROCm runtime itself reads) — no
// rocm-smi process spawn. Returns one dict per GPU node: gfx target, CU count, VRAM, PCI bus and
// a stable unique id.
static std::string read_file(const std::string& p) {
  std::ifstream f(p);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

std::vector<std::map<std::string, std::string>> detect_kfd_gpus(const std::string& root) {
  std::vector<std::map<std::string, std::string>> out;
  const std::string nodes = root + "/sys/class/kfd/kfd/topology/nodes";
  DIR* d = opendir(nodes.c_str());
  if (!d) return out;
  std::vector<int> ids;
  while (dirent* e = readdir(d)) {
    if (e->d_name[0] == '.') continue;
    ids.push_back(std::atoi(e->d_name));
  }
  closedir(d);
  std::sort(ids.begin(), ids.end());
  int gpu_index = 0;
  for (int id : ids) {
    const std::string base = nodes + "/" + std::to_string(id);
    std::istringstream props(read_file(base + "/properties"));
    std::map<std::string, std::string> kv;
    std::string k, v;
    while (props >> k >> v) kv[k] = v;
    if (kv["simd_count"].empty() || kv["simd_count"] == "0") continue;  // CPU node
    std::map<std::string, std::string> g;
    g["index"] = std::to_string(gpu_index++);
    g["node_id"] = std::to_string(id);
    const long ver = std::atol(kv["gfx_target_version"].c_str());
    char buf[32];
    snprintf(buf, sizeof(buf), "gfx%ld%ld%lx", ver / 10000, (ver / 100) % 100, ver % 100);
    g["gfx_target"] = buf;
    g["simd_count"] = kv["simd_count"];
    g["cu_count"] = std::to_string(std::atol(kv["simd_count"].c_str()) /
                                   std::max(1L, std::atol(kv["simd_per_cu"].c_str())));
    g["unique_id"] = kv["unique_id"];
    g["location_id"] = kv["location_id"];
    g["domain"] = kv["domain"];  // PCI domain: with location_id, the device's PCI address
    g["drm_render_minor"] = kv["drm_render_minor"];
    g["vendor_id"] = kv["vendor_id"];
    g["device_id"] = kv["device_id"];
    std::istringstream mem(read_file(base + "/mem_banks/0/properties"));
    std::map<std::string, std::string> mkv;
    while (mem >> k >> v) mkv[k] = v;
    g["vram_bytes"] = mkv["size_in_bytes"];
    out.push_back(g);
  }
  return out;
}

}  // namespace dca_native

PYBIND11_MODULE(_native, m) {
  using namespace dca_native;
  m.doc() = "determined_clone_amd native runtime: scheduler + device detection";
  py::class_<Agent>(m, "Agent")
      .def(py::init<>())
      .def_readwrite("id", &Agent::id)
      .def_readwrite("num_slots", &Agent::num_slots)
      .def_readwrite("slot_owner", &Agent::slot_owner)
      .def_readwrite("slot_enabled", &Agent::slot_enabled)
      .def_readwrite("enabled", &Agent::enabled)
      .def_readwrite("pool", &Agent::pool)
      .def_readwrite("label", &Agent::label)
      .def_readwrite("max_zero_slot", &Agent::max_zero_slot)
      .def_readwrite("zero_slot_used", &Agent::zero_slot_used);
  py::class_<Request>(m, "Request")
      .def(py::init<>())
      .def_readwrite("alloc_id", &Request::alloc_id)
      .def_readwrite("job_id", &Request::job_id)
      .def_readwrite("slots", &Request::slots)
      .def_readwrite("priority", &Request::priority)
      .def_readwrite("weight", &Request::weight)
      .def_readwrite("submit_time", &Request::submit_time)
      .def_readwrite("job_position", &Request::job_position)
      .def_readwrite("preemptible", &Request::preemptible)
      .def_readwrite("pool", &Request::pool)
      .def_readwrite("label", &Request::label)
      .def_readwrite("blocked_agents", &Request::blocked_agents)
      .def_readwrite("max_slots", &Request::max_slots)
      .def_readwrite("job_submit_time", &Request::job_submit_time);
  py::class_<Running>(m, "Running")
      .def(py::init<>())
      .def_readwrite("alloc_id", &Running::alloc_id)
      .def_readwrite("job_id", &Running::job_id)
      .def_readwrite("slots", &Running::slots)
      .def_readwrite("priority", &Running::priority)
      .def_readwrite("weight", &Running::weight)
      .def_readwrite("start_time", &Running::start_time)
      .def_readwrite("preemptible", &Running::preemptible)
      .def_readwrite("max_slots", &Running::max_slots)
      .def_readwrite("submit_time", &Running::submit_time)
      .def_readwrite("job_submit_time", &Running::job_submit_time)
      .def_readwrite("job_position", &Running::job_position)
      .def_readwrite("agents", &Running::agents);
  py::class_<Placement>(m, "Placement")
      .def(py::init<>())
      .def_readwrite("agent_id", &Placement::agent_id)
      .def_readwrite("slots", &Placement::slots);
  py::class_<Decision>(m, "Decision")
      .def_readonly("start", &Decision::start)
      .def_readonly("preempt", &Decision::preempt);
  py::class_<Scheduler>(m, "Scheduler")
      .def(py::init<std::string, std::string, bool>(), py::arg("policy") = "priority",
           py::arg("fit") = "best", py::arg("preemption") = true)
      .def("schedule", &Scheduler::schedule, py::call_guard<py::gil_scoped_release>());
  m.def("find_fit", &find_fit);
  m.def("detect_kfd_gpus", &detect_kfd_gpus, py::arg("root") = "");
}
