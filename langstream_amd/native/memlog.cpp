// In-process partitioned topic log ("memory" streaming cluster).
//
// Parity target: the broker semantics the reference relies on through Kafka
// (KAFKA/KafkaStreamingClusterRuntime.java:41-88, KRT/KafkaConsumerWrapper.java:70-277,
// KRT/KafkaReaderWrapper.java:60-150): partitioned append-only topics, consumer groups
// sharing partitions (replica data-parallelism), out-of-order acknowledgement with a
// committed offset that only advances through the contiguous prefix, at-least-once
// redelivery from the committed offset after a rebalance, and group-less readers that
// start at earliest / latest / an absolute per-partition offset.
//
// Messages are Python objects held by reference (no serialisation on the in-process
// hot path).  Concurrency: every method is entered with the GIL held and the GIL is
// the data lock (so Python refcounts are never touched without it); blocking reads
// drop the GIL and sleep on a condition variable keyed by an append sequence number,
// which is the only state guarded by `cvmu_` -- no thread ever waits for the GIL
// while holding `cvmu_`, so the two locks cannot deadlock.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace {

// Interpreter-exit gate.  A daemon reader parked in wait_for() (GIL released) when
// CPython finalizes is ended with pthread_exit as it re-takes the GIL; that forced unwind
// through pybind11 frames holding py::objects aborts the process.  shutdown_waiters()
// (called from an atexit hook) closes the gate: parked waiters wake within one slice and
// later calls return at once without dropping the GIL.
std::atomic<bool> g_closing{false};
std::atomic<int> g_waiters{0};
constexpr auto kWaitSlice = std::chrono::milliseconds(20);

struct Partition {
  std::deque<py::object> msgs;  // msgs[i] has offset base + i
  int64_t base = 0;
  int64_t end() const { return base + (int64_t)msgs.size(); }
};

struct GroupPartState {
  int64_t committed = 0;        // next offset to (re)deliver after a rebalance
  std::set<int64_t> done;       // acknowledged offsets >= committed
  int64_t position = 0;         // next offset to hand out to the current owner
  std::string owner;
};

struct Group {
  std::vector<std::string> members;  // join order
  std::vector<GroupPartState> parts;
  int64_t generation = 0;
};

struct Topic {
  std::vector<Partition> parts;
  std::unordered_map<std::string, Group> groups;
  int64_t total = 0;
  int64_t retention = 0;  // max messages per partition kept (0 = unbounded)
};

class MemLog {
 public:
  void create_topic(const std::string& name, int partitions, int64_t retention) {
    if (topics_.count(name)) return;
    auto t = std::make_unique<Topic>();
    t->parts.resize(std::max(1, partitions));
    t->retention = retention;
    topics_[name] = std::move(t);
  }

  bool has_topic(const std::string& name) {
    return topics_.count(name) > 0;
  }

  void delete_topic(const std::string& name) {
    auto it = topics_.find(name);
    if (it == topics_.end()) return;
    topics_.erase(it);
    notify();
  }

  std::vector<std::string> topics() {
    std::vector<std::string> r;
    for (auto& kv : topics_) r.push_back(kv.first);
    return r;
  }

  int partitions(const std::string& name) {
    return (int)get(name)->parts.size();
  }

  // Append; partition < 0 -> hash of `key_hash` (caller computes) modulo partitions.
  std::pair<int, int64_t> append(const std::string& name, py::object msg, int64_t key_hash, int partition) {
    std::pair<int, int64_t> r;
    {
        Topic* t = get(name);
      const int np = (int)t->parts.size();
      int p = partition >= 0 ? partition % np : (int)((uint64_t)key_hash % (uint64_t)np);
      Partition& part = t->parts[p];
      const int64_t off = part.end();
      part.msgs.push_back(std::move(msg));
      t->total++;
      if (t->retention > 0) {
        while ((int64_t)part.msgs.size() > t->retention) {
          part.msgs.pop_front();
          part.base++;
        }
      }
      r = {p, off};
    }
    notify();
    return r;
  }

  // --- consumer groups --------------------------------------------------------
  void join(const std::string& name, const std::string& group, const std::string& member) {
    Topic* t = get(name);
    Group& gr = t->groups[group];
    if (gr.parts.empty()) gr.parts.resize(t->parts.size());
    if (std::find(gr.members.begin(), gr.members.end(), member) == gr.members.end()) gr.members.push_back(member);
    rebalance(gr);
  }

  void leave(const std::string& name, const std::string& group, const std::string& member) {
    {
        auto it = topics_.find(name);
      if (it == topics_.end()) return;
      auto git = it->second->groups.find(group);
      if (git == it->second->groups.end()) return;
      auto& m = git->second.members;
      m.erase(std::remove(m.begin(), m.end(), member), m.end());
      rebalance(git->second);
    }
    notify();
  }

  std::vector<int> assignment(const std::string& name, const std::string& group, const std::string& member) {
    Topic* t = get(name);
    auto& gr = t->groups[group];
    std::vector<int> r;
    for (size_t p = 0; p < gr.parts.size(); ++p)
      if (gr.parts[p].owner == member) r.push_back((int)p);
    return r;
  }

  // Poll up to max_records from the member's partitions, waiting up to timeout_ms.
  // Returns list of (partition, offset, msg).
  py::list poll(const std::string& name, const std::string& group, const std::string& member, int max_records,
                double timeout_ms) {
    py::list out;
    const auto deadline =
        std::chrono::steady_clock::now() + std::chrono::microseconds((int64_t)(timeout_ms * 1000));
    while (true) {
      const uint64_t s0 = seq();
      auto it = topics_.find(name);
      if (it == topics_.end()) break;
      Topic* t = it->second.get();
      auto git = t->groups.find(group);
      if (git == t->groups.end()) break;
      Group& gr = git->second;
      const size_t np = gr.parts.size();
      int n = 0;
      // round-robin over the owned partitions starting at a rotating index
      for (size_t k = 0; k < np && n < max_records; ++k) {
        const size_t p = (rr_ + k) % np;
        GroupPartState& st = gr.parts[p];
        if (st.owner != member) continue;
        Partition& part = t->parts[p];
        if (st.position < part.base) st.position = part.base;  // evicted by retention
        while (st.position < part.end() && n < max_records) {
          out.append(py::make_tuple((int)p, st.position, part.msgs[st.position - part.base]));
          st.position++;
          n++;
        }
      }
      rr_++;
      if (n > 0 || !wait_for(s0, deadline)) break;
    }
    return out;
  }

  // Acknowledge offsets; the committed offset advances through the contiguous prefix
  // of acknowledged offsets (KafkaConsumerWrapper.java:203-277 semantics).
  std::map<int, int64_t> ack(const std::string& name, const std::string& group,
                             const std::vector<std::pair<int, int64_t>>& offsets) {
    Topic* t = get(name);
    Group& gr = t->groups[group];
    if (gr.parts.empty()) gr.parts.resize(t->parts.size());
    std::map<int, int64_t> res;
    for (auto& po : offsets) {
      if (po.first < 0 || po.first >= (int)gr.parts.size()) continue;
      GroupPartState& st = gr.parts[po.first];
      if (po.second < st.committed) continue;
      st.done.insert(po.second);
      while (!st.done.empty() && *st.done.begin() == st.committed) {
        st.done.erase(st.done.begin());
        st.committed++;
      }
      res[po.first] = st.committed;
    }
    return res;
  }

  std::vector<int64_t> committed(const std::string& name, const std::string& group) {
    Topic* t = get(name);
    auto git = t->groups.find(group);
    std::vector<int64_t> r(t->parts.size(), 0);
    if (git == t->groups.end()) return r;
    for (size_t p = 0; p < git->second.parts.size(); ++p) r[p] = git->second.parts[p].committed;
    return r;
  }

  // Total messages not yet committed by the group (lag).
  int64_t lag(const std::string& name, const std::string& group) {
    Topic* t = get(name);
    auto git = t->groups.find(group);
    int64_t lag = 0;
    for (size_t p = 0; p < t->parts.size(); ++p) {
      const int64_t c = (git == t->groups.end()) ? t->parts[p].base : git->second.parts[p].committed;
      lag += t->parts[p].end() - std::max(c, t->parts[p].base);
    }
    return lag;
  }

  // --- group-less readers -----------------------------------------------------
  std::vector<int64_t> end_offsets(const std::string& name) {
    Topic* t = get(name);
    std::vector<int64_t> r;
    for (auto& p : t->parts) r.push_back(p.end());
    return r;
  }

  std::vector<int64_t> begin_offsets(const std::string& name) {
    Topic* t = get(name);
    std::vector<int64_t> r;
    for (auto& p : t->parts) r.push_back(p.base);
    return r;
  }

  // Read from explicit per-partition positions (updated in place); waits up to timeout.
  py::tuple read_from(const std::string& name, std::vector<int64_t> positions, int max_records, double timeout_ms) {
    py::list out;
    const auto deadline =
        std::chrono::steady_clock::now() + std::chrono::microseconds((int64_t)(timeout_ms * 1000));
    while (true) {
      const uint64_t s0 = seq();
      auto it = topics_.find(name);
      if (it == topics_.end()) break;
      Topic* t = it->second.get();
      if (positions.size() < t->parts.size()) positions.resize(t->parts.size(), 0);
      int n = 0;
      for (size_t p = 0; p < t->parts.size() && n < max_records; ++p) {
        Partition& part = t->parts[p];
        if (positions[p] < part.base) positions[p] = part.base;
        while (positions[p] < part.end() && n < max_records) {
          out.append(py::make_tuple((int)p, positions[p], part.msgs[positions[p] - part.base]));
          positions[p]++;
          n++;
        }
      }
      if (n > 0 || !wait_for(s0, deadline)) break;
    }
    return py::make_tuple(out, positions);
  }

  int64_t total(const std::string& name) {
    return get(name)->total;
  }

  void wakeup() { notify(); }

 private:
  uint64_t seq() {
    std::lock_guard<std::mutex> g(cvmu_);
    return seq_;
  }
  void notify() {
    {
      std::lock_guard<std::mutex> g(cvmu_);
      seq_++;
    }
    cv_.notify_all();
  }
  // Sleep (GIL released) until an append/rebalance bumps the sequence or the deadline
  // passes.  Returns false on timeout.
  // Sleep (GIL released) in short slices until an append/rebalance bumps the sequence,
  // the deadline passes or the exit gate closes.  Returns false on timeout.
  bool wait_for(uint64_t s0, std::chrono::steady_clock::time_point deadline) {
    if (g_closing.load()) return false;
    g_waiters++;
    bool woke = false;
    {
      py::gil_scoped_release nogil;
      std::unique_lock<std::mutex> lk(cvmu_);
      while (!woke && !g_closing.load()) {
        auto now = std::chrono::steady_clock::now();
        if (now >= deadline) break;
        woke = cv_.wait_until(lk, std::min(deadline, now + kWaitSlice), [&] { return seq_ != s0; });
      }
    }
    g_waiters--;
    return woke;
  }

  Topic* get(const std::string& name) {
    auto it = topics_.find(name);
    if (it == topics_.end()) throw std::runtime_error("topic does not exist: " + name);
    return it->second.get();
  }

  // Range-assign partitions to members in join order; ownership changes reset the
  // delivery position to the committed offset (at-least-once redelivery).
  static void rebalance(Group& gr) {
    gr.generation++;
    const size_t np = gr.parts.size(), nm = gr.members.size();
    for (size_t p = 0; p < np; ++p) {
      std::string owner = nm ? gr.members[p % nm] : std::string();
      GroupPartState& st = gr.parts[p];
      if (st.owner != owner) {
        st.owner = owner;
        st.position = st.committed;
        st.done.clear();
      }
    }
  }

  std::mutex cvmu_;
  std::condition_variable cv_;
  uint64_t seq_ = 0;
  std::unordered_map<std::string, std::unique_ptr<Topic>> topics_;
  size_t rr_ = 0;
};

}  // namespace

void bind_memlog(py::module_& m) {
  py::class_<MemLog, std::shared_ptr<MemLog>>(m, "MemLog")
      .def(py::init<>())
      .def("create_topic", &MemLog::create_topic, py::arg("name"), py::arg("partitions") = 1,
           py::arg("retention") = 0)
      .def("has_topic", &MemLog::has_topic)
      .def("delete_topic", &MemLog::delete_topic)
      .def("topics", &MemLog::topics)
      .def("partitions", &MemLog::partitions)
      .def("append", &MemLog::append, py::arg("name"), py::arg("msg"), py::arg("key_hash") = 0,
           py::arg("partition") = -1)
      .def("join", &MemLog::join)
      .def("leave", &MemLog::leave)
      .def("assignment", &MemLog::assignment)
      .def("poll", &MemLog::poll, py::arg("name"), py::arg("group"), py::arg("member"), py::arg("max_records") = 500,
           py::arg("timeout_ms") = 1000.0)
      .def("ack", &MemLog::ack)
      .def("committed", &MemLog::committed)
      .def("lag", &MemLog::lag)
      .def("end_offsets", &MemLog::end_offsets)
      .def("begin_offsets", &MemLog::begin_offsets)
      .def("read_from", &MemLog::read_from, py::arg("name"), py::arg("positions"), py::arg("max_records") = 500,
           py::arg("timeout_ms") = 1000.0)
      .def("total", &MemLog::total)
      .def("wakeup", &MemLog::wakeup);
  m.def("memlog_close_gate", [] { g_closing.store(true); });
  m.def("memlog_waiters", [] { return g_waiters.load(); });
}
