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
  int job_position = 0;  // user re-ordering within the queue (UpdateJobQueue)
  bool preemptible = true;
  std::string pool;
  std::string label;
  std::vector<std::string> blocked_agents;
};

struct Running {
  std::string alloc_id;
  std::string job_id;
  int slots = 0;
  int priority = 42;
  double weight = 1.0;
  double start_time = 0.0;
  bool preemptible = true;
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

  Decision priority(std::vector<Agent>& agents, std::vector<Request>& pending,
                    std::vector<Running>& running) {
    Decision d;
    std::sort(pending.begin(), pending.end(), req_order);
    // Zero-slot and slot tasks are scheduled independently.
    for (int zero = 0; zero < 2; ++zero) {
      std::map<int, std::vector<Request*>> by_prio;
      for (auto& r : pending)
        if ((r.slots == 0) == (zero == 1)) by_prio[r.priority].push_back(&r);
      bool backfilling = false;
      std::set<std::string> to_release;
      for (auto& kv : by_prio) {
        std::vector<Request*> failed;
        for (Request* r : kv.second) {
          auto ps = find_fit(*r, agents, fit_);
          if (ps.empty()) {
            failed.push_back(r);
            continue;
          }
          const bool allowed = to_release.empty() && (!backfilling || (preemption_ && r->preemptible));
          if (allowed) {
            apply(agents, r->alloc_id, ps);
            d.start.emplace_back(r->alloc_id, ps);
          }
        }
        if (!failed.empty()) backfilling = true;
        if (!preemption_) continue;
        for (Request* r : failed) {
          // Victims: lower-priority (larger number), preemptible, newest first.
          std::vector<Running*> victims;
          for (auto& run : running)
            if (run.priority > r->priority && run.preemptible && !to_release.count(run.alloc_id) &&
                (run.slots == 0) == (r->slots == 0))
              victims.push_back(&run);
          std::sort(victims.begin(), victims.end(), [](Running* a, Running* b) {
            if (a->priority != b->priority) return a->priority > b->priority;
            return a->start_time > b->start_time;
          });
          std::vector<Agent> trial = agents;
          std::vector<std::string> chosen;
          bool placed = false;
          for (Running* v : victims) {
            release(trial, v->alloc_id, 0);
            chosen.push_back(v->alloc_id);
            if (!find_fit(*r, trial, fit_).empty()) {
              placed = true;
              break;
            }
          }
          if (placed)
            for (auto& c : chosen) to_release.insert(c);
        }
      }
      for (auto& a : to_release) d.preempt.push_back(a);
    }
    return d;
  }

  Decision fair_share(std::vector<Agent>& agents, std::vector<Request>& pending,
                      std::vector<Running>& running) {
    Decision d;
    int capacity = 0;
    for (auto& a : agents)
      if (a.enabled) capacity += a.usable_slots();
    struct Group {
      double weight = 1.0;
      int running = 0;
      int demand = 0;
      double share = 0;
      std::vector<Request*> pend;
      std::vector<Running*> run;
    };
    std::map<std::string, Group> groups;
    for (auto& r : running) {
      auto& g = groups[r.job_id];
      g.weight = r.weight;
      g.running += r.slots;
      g.demand += r.slots;
      g.run.push_back(&r);
    }
    for (auto& r : pending) {
      auto& g = groups[r.job_id];
      g.weight = r.weight;
      g.demand += r.slots;
      g.pend.push_back(&r);
    }
    // Water-filling: groups demanding less than their weighted share keep their demand; the
    // remaining capacity is re-split among the rest by weight.
    std::vector<std::string> open;
    for (auto& kv : groups) open.push_back(kv.first);
    double left = capacity;
    while (!open.empty()) {
      double wsum = 0;
      for (auto& id : open) wsum += groups[id].weight;
      bool changed = false;
      std::vector<std::string> still;
      for (auto& id : open) {
        auto& g = groups[id];
        const double fair = wsum > 0 ? left * g.weight / wsum : 0;
        if (g.demand <= fair) {
          g.share = g.demand;
          changed = true;
        } else {
          still.push_back(id);
        }
      }
      if (!changed) {
        for (auto& id : still) groups[id].share = wsum > 0 ? left * groups[id].weight / wsum : 0;
        break;
      }
      left = capacity;
      for (auto& kv : groups)
        if (std::find(still.begin(), still.end(), kv.first) == still.end()) left -= kv.second.share;
      open = still;
    }
    // Start tasks of under-share groups, most-starved first.
    std::vector<std::string> order;
    for (auto& kv : groups) order.push_back(kv.first);
    std::sort(order.begin(), order.end(), [&](const std::string& a, const std::string& b) {
      const double ra = groups[a].share > 0 ? groups[a].running / groups[a].share : 1e9;
      const double rb = groups[b].share > 0 ? groups[b].running / groups[b].share : 1e9;
      return ra != rb ? ra < rb : a < b;
    });
    bool starved = false;
    for (auto& id : order) {
      auto& g = groups[id];
      std::sort(g.pend.begin(), g.pend.end(), [](Request* a, Request* b) { return req_order(*a, *b); });
      for (Request* r : g.pend) {
        if (g.running + r->slots > std::ceil(g.share - 1e-9) && g.running > 0) {
          starved = true;
          break;
        }
        auto ps = find_fit(*r, agents, fit_);
        if (ps.empty()) {
          starved = true;
          break;
        }
        apply(agents, r->alloc_id, ps);
        d.start.emplace_back(r->alloc_id, ps);
        g.running += r->slots;
      }
    }
    // Preempt newest allocations of groups above their share while someone is starved.
    if (starved && preemption_) {
      for (auto& kv : groups) {
        auto& g = kv.second;
        std::sort(g.run.begin(), g.run.end(), [](Running* a, Running* b) { return a->start_time > b->start_time; });
        int over = g.running - static_cast<int>(std::floor(g.share + 1e-9));
        for (Running* r : g.run) {
          if (over <= 0) break;
          if (!r->preemptible) continue;
          d.preempt.push_back(r->alloc_id);
          over -= r->slots;
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
      .def_readwrite("blocked_agents", &Request::blocked_agents);
  py::class_<Running>(m, "Running")
      .def(py::init<>())
      .def_readwrite("alloc_id", &Running::alloc_id)
      .def_readwrite("job_id", &Running::job_id)
      .def_readwrite("slots", &Running::slots)
      .def_readwrite("priority", &Running::priority)
      .def_readwrite("weight", &Running::weight)
      .def_readwrite("start_time", &Running::start_time)
      .def_readwrite("preemptible", &Running::preemptible);
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
