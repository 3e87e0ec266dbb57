// Cross-process partitioned topic log in shared memory ("shm" streaming cluster).
//
// The broker of a single-node multi-GPU deployment: one OS process per GPU (the agent
// replicas of SURVEY §2.9 DP), all mapping the same file under /dev/shm.  It gives the
// replicas what the reference gets from Kafka (KAFKA/KafkaStreamingClusterRuntime.java:
// 41-88, KRT/KafkaConsumerWrapper.java:70-277, KRT/KafkaReaderWrapper.java:60-150):
//   * partitioned append-only topics;
//   * consumer groups shared across processes -- partitions are range-assigned over the
//     members in join order and re-assigned when a member joins, leaves or its process
//     dies (pid liveness), the new owner redelivering from the committed offset
//     (at-least-once);
//   * out-of-order acknowledgement kept by the owning consumer (a per-partition set, as
//     KafkaConsumerWrapper's TreeSet) with only the contiguous committed prefix
//     published to the shared group state;
//   * group-less readers at earliest / latest / absolute per-partition offsets.
//
// Layout: [Header | blocks...].  Each partition is a chain of fixed-size blocks taken
// from a free list; records are [u32 len | u32 pad | bytes] packed 8-byte aligned.
// Blocks are recycled oldest-first when the arena runs out, but only once every group
// of the topic has committed past them (producers otherwise back off and retry, i.e.
// backpressure), or -- for topics nobody consumes as a group -- unconditionally.
// Concurrency: one robust process-shared mutex guards all metadata and block contents;
// blocking reads sleep on a futex word bumped by every append / rebalance.  The GIL is
// released for every native section, so other Python threads keep running while a
// thread waits for the cross-process lock or for data.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <errno.h>
#include <fcntl.h>
#include <linux/futex.h>
#include <pthread.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

namespace py = pybind11;

namespace {

constexpr uint64_t kMagic = 0x4c53484d4c4f4731ull;  // "LSHMLOG1"
constexpr int kMaxTopics = 128;
constexpr int kMaxParts = 64;
constexpr int kMaxGroups = 256;
constexpr int kMaxMembers = 64;
constexpr int kNameLen = 128;
constexpr int kMemberLen = 64;
constexpr auto kWaitSlice = std::chrono::milliseconds(20);

std::atomic<bool> g_closing{false};
std::atomic<int> g_waiters{0};

struct PartMeta {
  int64_t base;    // first retained offset
  int64_t end;     // next offset to append
  int32_t head;    // oldest block (-1: none)
  int32_t tail;    // block being appended to
};

struct TopicMeta {
  char name[kNameLen];
  uint32_t used;
  int32_t nparts;
  int64_t retention;  // max messages kept per partition (0: bounded only by the arena)
  uint64_t total;
  uint64_t incarnation;
  PartMeta parts[kMaxParts];
};

struct MemberMeta {
  char id[kMemberLen];
  int32_t pid;
  uint32_t used;
};

struct GroupMeta {
  char name[kNameLen];
  int32_t topic;
  uint32_t used;
  uint64_t topic_incarnation;
  uint64_t generation;
  int32_t nmembers;
  int32_t pad;
  MemberMeta members[kMaxMembers];   // join order
  int64_t committed[kMaxParts];
  int32_t owner[kMaxParts];          // member slot, -1 none
  uint64_t owner_since[kMaxParts];   // generation at which the owner last changed
};

struct BlockHdr {
  int32_t next;
  int32_t topic;
  int32_t part;
  uint32_t count;
  uint64_t serial;
  int64_t base;   // offset of the first record
  uint64_t used;  // payload bytes used
  uint64_t pad[3];
};
static_assert(sizeof(BlockHdr) == 64, "block header");

struct Header {
  uint64_t magic;
  uint64_t size;
  uint64_t block_bytes;
  uint64_t blocks_off;
  int32_t nblocks;
  int32_t next_unused;   // blocks [next_unused, nblocks) never handed out yet
  int32_t free_head;
  int32_t nfree;
  uint64_t alloc_serial;
  uint64_t incarnations;
  pthread_mutex_t mu;
  alignas(64) std::atomic<uint32_t> seq;
  std::atomic<uint32_t> waiters;
  TopicMeta topics[kMaxTopics];
  GroupMeta groups[kMaxGroups];
};

inline int futex(std::atomic<uint32_t>* addr, int op, uint32_t val, const timespec* ts) {
  return (int)syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), op, val, ts, nullptr, 0);
}

inline bool pid_alive(int32_t pid) {
  if (pid <= 0) return false;
  return kill(pid, 0) == 0 || errno != ESRCH;
}

void copy_name(char* dst, const std::string& s, size_t cap) {
  if (s.size() >= cap) throw std::invalid_argument("name too long: " + s);
  std::memset(dst, 0, cap);
  std::memcpy(dst, s.data(), s.size());
}

struct Rec {
  int part;
  int64_t off;
  std::string data;
};

class ShmLog;

// RAII holder of the cross-process mutex (robust: a holder that died is recovered).
class Locked {
 public:
  explicit Locked(Header* h) : h_(h) {
    int r = pthread_mutex_lock(&h_->mu);
    if (r == EOWNERDEAD) pthread_mutex_consistent(&h_->mu);
    else if (r != 0) throw std::runtime_error("shm log: mutex lock failed");
  }
  ~Locked() { pthread_mutex_unlock(&h_->mu); }
  Locked(const Locked&) = delete;
  Locked& operator=(const Locked&) = delete;

 private:
  Header* h_;
};

class ShmLog : public std::enable_shared_from_this<ShmLog> {
 public:
  ShmLog(const std::string& path, uint64_t size, uint64_t block_bytes) : path_(path) {
    if (block_bytes < 4096 || (block_bytes & 7)) throw std::invalid_argument("block size must be >= 4096, 8-aligned");
    const uint64_t hdr = (sizeof(Header) + 4095) & ~uint64_t(4095);
    if (size < hdr + 4 * block_bytes) throw std::invalid_argument("shm log too small for 4 blocks");
    bool creator = false;
    int fd = open(path.c_str(), O_RDWR | O_CREAT | O_EXCL, 0600);
    if (fd >= 0) {
      creator = true;
      if (ftruncate(fd, (off_t)size) != 0) {
        close(fd);
        unlink(path.c_str());
        throw std::runtime_error("shm log: ftruncate failed for " + path);
      }
    } else {
      if (errno != EEXIST) throw std::runtime_error("shm log: cannot create " + path + ": " + strerror(errno));
      fd = open(path.c_str(), O_RDWR);
      if (fd < 0) throw std::runtime_error("shm log: cannot open " + path + ": " + strerror(errno));
      // wait for the creator to size the file
      for (int i = 0; i < 5000; ++i) {
        struct stat st;
        if (fstat(fd, &st) == 0 && (uint64_t)st.st_size >= hdr) {
          size = (uint64_t)st.st_size;
          break;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
      }
    }
    void* p = mmap(nullptr, size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) throw std::runtime_error("shm log: mmap failed for " + path);
    base_ = static_cast<char*>(p);
    size_ = size;
    h_ = reinterpret_cast<Header*>(base_);
    if (creator) {
      std::memset(h_, 0, sizeof(Header));
      h_->size = size;
      h_->block_bytes = block_bytes;
      h_->blocks_off = hdr;
      h_->nblocks = (int32_t)((size - hdr) / block_bytes);
      h_->free_head = -1;
      pthread_mutexattr_t a;
      pthread_mutexattr_init(&a);
      pthread_mutexattr_setpshared(&a, PTHREAD_PROCESS_SHARED);
      pthread_mutexattr_setrobust(&a, PTHREAD_MUTEX_ROBUST);
      pthread_mutex_init(&h_->mu, &a);
      pthread_mutexattr_destroy(&a);
      std::atomic_thread_fence(std::memory_order_release);
      reinterpret_cast<std::atomic<uint64_t>*>(&h_->magic)->store(kMagic, std::memory_order_release);
    } else {
      for (int i = 0; i < 10000; ++i) {
        if (reinterpret_cast<std::atomic<uint64_t>*>(&h_->magic)->load(std::memory_order_acquire) == kMagic) break;
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
      }
      if (h_->magic != kMagic) throw std::runtime_error("shm log: " + path + " is not an initialised log");
    }
  }

  ~ShmLog() {
    if (base_) munmap(base_, size_);
  }

  const std::string& path() const { return path_; }
  uint64_t max_record() const { return h_->block_bytes - sizeof(BlockHdr) - 8; }

  void unlink_file() { ::unlink(path_.c_str()); }

  // --- topics ---------------------------------------------------------------------
  void create_topic(const std::string& name, int partitions, int64_t retention) {
    if (partitions > kMaxParts) throw std::invalid_argument("at most 64 partitions per topic");
    Locked l(h_);
    if (find_topic(name) >= 0) return;
    for (int i = 0; i < kMaxTopics; ++i) {
      TopicMeta& t = h_->topics[i];
      if (t.used) continue;
      std::memset(&t, 0, sizeof(TopicMeta));
      copy_name(t.name, name, kNameLen);
      t.nparts = std::max(1, partitions);
      t.retention = retention;
      t.incarnation = ++h_->incarnations;
      for (int p = 0; p < kMaxParts; ++p) t.parts[p] = PartMeta{0, 0, -1, -1};
      t.used = 1;
      return;
    }
    throw std::runtime_error("shm log: too many topics");
  }

  bool has_topic(const std::string& name) {
    Locked l(h_);
    return find_topic(name) >= 0;
  }

  void delete_topic(const std::string& name) {
    {
      Locked l(h_);
      int ti = find_topic(name);
      if (ti < 0) return;
      TopicMeta& t = h_->topics[ti];
      for (int p = 0; p < t.nparts; ++p) {
        int32_t b = t.parts[p].head;
        while (b >= 0) {
          int32_t nx = blk(b)->next;
          free_block(b);
          b = nx;
        }
      }
      for (int g = 0; g < kMaxGroups; ++g)
        if (h_->groups[g].used && h_->groups[g].topic == ti) h_->groups[g].used = 0;
      t.used = 0;
    }
    notify();
  }

  std::vector<std::string> topics() {
    Locked l(h_);
    std::vector<std::string> r;
    for (int i = 0; i < kMaxTopics; ++i)
      if (h_->topics[i].used) r.emplace_back(h_->topics[i].name);
    return r;
  }

  int partitions(const std::string& name) {
    Locked l(h_);
    return topic(name).nparts;
  }

  // Append one record; partition < 0 -> key_hash modulo partitions.  Blocks (GIL
  // released) while the arena is full of uncommitted data, up to `timeout_ms`.
  std::pair<int, int64_t> append(const std::string& name, const std::string& data, int64_t key_hash, int partition,
                                 double timeout_ms) {
    if (data.size() > max_record())
      throw std::invalid_argument("record of " + std::to_string(data.size()) + " bytes exceeds the shm block size");
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::microseconds((int64_t)(timeout_ms * 1000));
    while (true) {
      int p = 0;
      int64_t off = -1;
      {
        Locked l(h_);
        int ti = find_topic(name);
        if (ti < 0) throw std::runtime_error("topic does not exist: " + name);
        TopicMeta& t = h_->topics[ti];
        p = partition >= 0 ? partition % t.nparts : (int)((uint64_t)key_hash % (uint64_t)t.nparts);
        off = try_append(ti, p, data);
      }
      if (off >= 0) {
        notify();
        return {p, off};
      }
      if (std::chrono::steady_clock::now() >= deadline)
        throw std::runtime_error("shm log full: every block holds uncommitted records (" + path_ + ")");
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
  }

  std::vector<int64_t> end_offsets(const std::string& name) {
    Locked l(h_);
    TopicMeta& t = topic(name);
    std::vector<int64_t> r;
    for (int p = 0; p < t.nparts; ++p) r.push_back(t.parts[p].end);
    return r;
  }

  std::vector<int64_t> begin_offsets(const std::string& name) {
    Locked l(h_);
    TopicMeta& t = topic(name);
    std::vector<int64_t> r;
    for (int p = 0; p < t.nparts; ++p) r.push_back(t.parts[p].base);
    return r;
  }

  int64_t total(const std::string& name) {
    Locked l(h_);
    return (int64_t)topic(name).total;
  }

  std::vector<int64_t> committed(const std::string& name, const std::string& group) {
    Locked l(h_);
    int ti = find_topic(name);
    if (ti < 0) throw std::runtime_error("topic does not exist: " + name);
    std::vector<int64_t> r(h_->topics[ti].nparts, 0);
    int gi = find_group(ti, group);
    if (gi >= 0)
      for (int p = 0; p < h_->topics[ti].nparts; ++p) r[p] = h_->groups[gi].committed[p];
    return r;
  }

  int64_t lag(const std::string& name, const std::string& group) {
    Locked l(h_);
    int ti = find_topic(name);
    if (ti < 0) throw std::runtime_error("topic does not exist: " + name);
    TopicMeta& t = h_->topics[ti];
    int gi = find_group(ti, group);
    int64_t lag = 0;
    for (int p = 0; p < t.nparts; ++p) {
      int64_t c = gi >= 0 ? h_->groups[gi].committed[p] : t.parts[p].base;
      lag += t.parts[p].end - std::max(c, t.parts[p].base);
    }
    return lag;
  }

  int group_members(const std::string& name, const std::string& group) {
    Locked l(h_);
    int ti = find_topic(name);
    if (ti < 0) return 0;
    int gi = find_group(ti, group);
    if (gi < 0) return 0;
    GroupMeta& g = h_->groups[gi];
    reap(g, h_->topics[ti].nparts);
    return g.nmembers;
  }

  // (topic, group, live members, committed offsets) of every group
  std::vector<std::tuple<std::string, std::string, int, std::vector<int64_t>>> groups() {
    Locked l(h_);
    std::vector<std::tuple<std::string, std::string, int, std::vector<int64_t>>> r;
    for (int i = 0; i < kMaxGroups; ++i) {
      GroupMeta& g = h_->groups[i];
      if (!g.used || !h_->topics[g.topic].used || g.topic_incarnation != h_->topics[g.topic].incarnation) continue;
      TopicMeta& t = h_->topics[g.topic];
      r.emplace_back(std::string(t.name), std::string(g.name), g.nmembers,
                     std::vector<int64_t>(g.committed, g.committed + t.nparts));
    }
    return r;
  }

  py::dict stats() {
    Locked l(h_);
    py::dict d;
    d["blocks"] = h_->nblocks;
    d["block_bytes"] = h_->block_bytes;
    d["free_blocks"] = h_->nfree + (h_->nblocks - h_->next_unused);
    int ng = 0, nt = 0;
    for (int i = 0; i < kMaxGroups; ++i) ng += h_->groups[i].used ? 1 : 0;
    for (int i = 0; i < kMaxTopics; ++i) nt += h_->topics[i].used ? 1 : 0;
    d["groups"] = ng;
    d["topics"] = nt;
    return d;
  }

  void wakeup() { notify(); }

  // --- internals shared with consumers/readers ------------------------------------
  Header* h() { return h_; }

  BlockHdr* blk(int32_t i) {
    return reinterpret_cast<BlockHdr*>(base_ + h_->blocks_off + (uint64_t)i * h_->block_bytes);
  }
  char* blk_data(int32_t i) { return reinterpret_cast<char*>(blk(i)) + sizeof(BlockHdr); }

  int find_topic(const std::string& name) {
    for (int i = 0; i < kMaxTopics; ++i)
      if (h_->topics[i].used && name == h_->topics[i].name) return i;
    return -1;
  }

  TopicMeta& topic(const std::string& name) {
    int i = find_topic(name);
    if (i < 0) throw std::runtime_error("topic does not exist: " + name);
    return h_->topics[i];
  }

  int find_group(int ti, const std::string& group) {
    for (int i = 0; i < kMaxGroups; ++i) {
      GroupMeta& g = h_->groups[i];
      if (g.used && g.topic == ti && g.topic_incarnation == h_->topics[ti].incarnation && group == g.name) return i;
    }
    return -1;
  }

  int ensure_group(int ti, const std::string& group) {
    int gi = find_group(ti, group);
    if (gi >= 0) return gi;
    for (int i = 0; i < kMaxGroups; ++i) {
      GroupMeta& g = h_->groups[i];
      if (g.used) continue;
      std::memset(&g, 0, sizeof(GroupMeta));
      copy_name(g.name, group, kNameLen);
      g.topic = ti;
      g.topic_incarnation = h_->topics[ti].incarnation;
      for (int p = 0; p < kMaxParts; ++p) {
        g.owner[p] = -1;
        g.committed[p] = h_->topics[ti].parts[p].base;
      }
      g.used = 1;
      return i;
    }
    throw std::runtime_error("shm log: too many consumer groups");
  }

  // Range-assign partitions over live members in join order.
  void rebalance(GroupMeta& g, int nparts) {
    g.generation++;
    std::vector<int> live;
    for (int m = 0; m < kMaxMembers; ++m)
      if (g.members[m].used) live.push_back(m);
    std::sort(live.begin(), live.end(), [&](int a, int b) { return a < b; });
    for (int p = 0; p < nparts; ++p) {
      int owner = live.empty() ? -1 : live[p % live.size()];
      if (g.owner[p] != owner) {
        g.owner[p] = owner;
        g.owner_since[p] = g.generation;
      }
    }
  }

  // Drop members whose process is gone; returns true when the group changed.
  bool reap(GroupMeta& g, int nparts) {
    bool changed = false;
    for (int m = 0; m < kMaxMembers; ++m) {
      if (g.members[m].used && !pid_alive(g.members[m].pid)) {
        g.members[m].used = 0;
        g.nmembers--;
        changed = true;
      }
    }
    if (changed) rebalance(g, nparts);
    return changed;
  }

  // Walk to the record at `pos` in partition (ti, p); returns (block, byte offset) or (-1, 0).
  std::pair<int32_t, uint64_t> locate(PartMeta& pm, int64_t pos) {
    for (int32_t b = pm.head; b >= 0; b = blk(b)->next) {
      BlockHdr* bh = blk(b);
      if (pos < bh->base + (int64_t)bh->count) {
        uint64_t byte = 0;
        char* d = blk_data(b);
        for (int64_t k = bh->base; k < pos; ++k) {
          uint32_t len;
          std::memcpy(&len, d + byte, 4);
          byte += (8 + len + 7) & ~uint64_t(7);
        }
        return {b, byte};
      }
    }
    return {-1, 0};
  }

  // Copy records of one partition from `pos` (advanced) into `out`.  `cur` caches the
  // block/byte position of `pos` so sequential reads do not rescan a block.
  struct Cursor {
    int32_t blk = -1;
    uint64_t serial = 0;
    uint64_t byte = 0;
    int64_t pos = -1;
  };

  // First offset still stored in partition p (retention may have dropped older blocks).
  int64_t part_base(int ti, int p) const { return h_->topics[ti].parts[p].base; }

  int read_part(int ti, int p, int64_t& pos, Cursor& cur, int max_records, uint64_t& budget, std::vector<Rec>& out) {
    PartMeta& pm = h_->topics[ti].parts[p];
    if (pos < pm.base) pos = pm.base;
    if (pos >= pm.end) return 0;
    int32_t b;
    uint64_t byte;
    if (cur.blk >= 0 && cur.pos == pos && blk(cur.blk)->serial == cur.serial) {
      b = cur.blk;
      byte = cur.byte;
    } else {
      std::tie(b, byte) = locate(pm, pos);
      if (b < 0) return 0;
    }
    int n = 0;
    while (pos < pm.end && n < max_records && budget > 0 && b >= 0) {
      BlockHdr* bh = blk(b);
      if (pos >= bh->base + (int64_t)bh->count) {
        b = bh->next;
        byte = 0;
        continue;
      }
      char* d = blk_data(b);
      uint32_t len;
      std::memcpy(&len, d + byte, 4);
      out.push_back(Rec{p, pos, std::string(d + byte + 8, len)});
      byte += (8 + len + 7) & ~uint64_t(7);
      budget = budget > len ? budget - len : 0;
      pos++;
      n++;
    }
    cur.blk = b;
    cur.serial = b >= 0 ? blk(b)->serial : 0;
    cur.byte = byte;
    cur.pos = pos;
    return n;
  }

  uint32_t seq() { return h_->seq.load(std::memory_order_acquire); }

  void notify() {
    h_->seq.fetch_add(1, std::memory_order_acq_rel);
    if (h_->waiters.load(std::memory_order_acquire) > 0) futex(&h_->seq, FUTEX_WAKE, INT32_MAX, nullptr);
  }

  // Sleep (GIL already released by the caller) until the sequence moves, the deadline
  // passes or the exit gate closes.  Returns false on timeout.
  bool wait_for(uint32_t s0, std::chrono::steady_clock::time_point deadline) {
    if (g_closing.load()) return false;
    g_waiters++;
    h_->waiters.fetch_add(1);
    bool woke = false;
    while (!g_closing.load()) {
      if (h_->seq.load(std::memory_order_acquire) != s0) {
        woke = true;
        break;
      }
      auto now = std::chrono::steady_clock::now();
      if (now >= deadline) break;
      auto slice = std::min(std::chrono::duration_cast<std::chrono::nanoseconds>(deadline - now),
                            std::chrono::duration_cast<std::chrono::nanoseconds>(kWaitSlice));
      timespec ts{(time_t)(slice.count() / 1000000000), (long)(slice.count() % 1000000000)};
      futex(&h_->seq, FUTEX_WAIT, s0, &ts);
    }
    h_->waiters.fetch_sub(1);
    g_waiters--;
    return woke;
  }

 private:
  int32_t alloc_block() {
    if (h_->free_head >= 0) {
      int32_t b = h_->free_head;
      h_->free_head = blk(b)->next;
      h_->nfree--;
      return b;
    }
    if (h_->next_unused < h_->nblocks) return h_->next_unused++;
    return -1;
  }

  void free_block(int32_t b) {
    BlockHdr* bh = blk(b);
    bh->serial = 0;
    bh->next = h_->free_head;
    h_->free_head = b;
    h_->nfree++;
  }

  // Is the head block of (ti, p) free to drop: not the tail, and (for consumed topics)
  // every group has committed past it.
  bool evictable(int ti, int p) {
    PartMeta& pm = h_->topics[ti].parts[p];
    if (pm.head < 0 || pm.head == pm.tail) return false;
    BlockHdr* bh = blk(pm.head);
    const int64_t last = bh->base + (int64_t)bh->count;
    for (int g = 0; g < kMaxGroups; ++g) {
      GroupMeta& gm = h_->groups[g];
      if (gm.used && gm.topic == ti && gm.topic_incarnation == h_->topics[ti].incarnation && gm.committed[p] < last)
        return false;
    }
    return true;
  }

  void drop_head(int ti, int p) {
    PartMeta& pm = h_->topics[ti].parts[p];
    int32_t b = pm.head;
    BlockHdr* bh = blk(b);
    pm.head = bh->next;
    pm.base = bh->base + (int64_t)bh->count;
    free_block(b);
  }

  // Evict the globally oldest evictable head block; false when none is.
  bool evict_one() {
    int bt = -1, bp = -1;
    uint64_t best = UINT64_MAX;
    for (int ti = 0; ti < kMaxTopics; ++ti) {
      if (!h_->topics[ti].used) continue;
      for (int p = 0; p < h_->topics[ti].nparts; ++p) {
        PartMeta& pm = h_->topics[ti].parts[p];
        if (pm.head >= 0 && blk(pm.head)->serial < best && evictable(ti, p)) {
          best = blk(pm.head)->serial;
          bt = ti;
          bp = p;
        }
      }
    }
    if (bt < 0) return false;
    drop_head(bt, bp);
    return true;
  }

  int64_t try_append(int ti, int p, const std::string& data) {
    TopicMeta& t = h_->topics[ti];
    PartMeta& pm = t.parts[p];
    const uint64_t need = (8 + data.size() + 7) & ~uint64_t(7);
    const uint64_t cap = h_->block_bytes - sizeof(BlockHdr);
    if (pm.tail < 0 || blk(pm.tail)->used + need > cap) {
      int32_t b = alloc_block();
      while (b < 0 && evict_one()) b = alloc_block();
      if (b < 0) return -1;
      BlockHdr* bh = blk(b);
      bh->next = -1;
      bh->topic = ti;
      bh->part = p;
      bh->count = 0;
      bh->serial = ++h_->alloc_serial;
      bh->base = pm.end;
      bh->used = 0;
      if (pm.tail >= 0) blk(pm.tail)->next = b;
      else pm.head = b;
      pm.tail = b;
      if (pm.head == b) pm.base = pm.end;
    }
    BlockHdr* bh = blk(pm.tail);
    char* d = blk_data(pm.tail) + bh->used;
    const uint32_t len = (uint32_t)data.size();
    std::memcpy(d, &len, 4);
    std::memset(d + 4, 0, 4);
    std::memcpy(d + 8, data.data(), len);
    bh->used += need;
    bh->count++;
    const int64_t off = pm.end++;
    t.total++;
    if (t.retention > 0)
      while (pm.end - pm.base > t.retention && pm.head != pm.tail &&
             pm.end - (blk(pm.head)->base + (int64_t)blk(pm.head)->count) >= t.retention)
        drop_head(ti, p);
    return off;
  }

  std::string path_;
  char* base_ = nullptr;
  uint64_t size_ = 0;
  Header* h_ = nullptr;
};

// A consumer-group member (one per agent replica).  Delivery positions and the
// out-of-order ack sets are process-local; only committed offsets are shared.
class ShmConsumer {
 public:
  ShmConsumer(std::shared_ptr<ShmLog> log, std::string topic, std::string group, std::string member)
      : log_(std::move(log)), topic_(std::move(topic)), group_(std::move(group)), member_(std::move(member)) {
    if (member_.size() >= (size_t)kMemberLen) throw std::invalid_argument("member id too long");
  }

  void start() {
    py::gil_scoped_release nogil;
    {
      Locked l(log_->h());
      int ti = log_->find_topic(topic_);
      if (ti < 0) throw std::runtime_error("topic does not exist: " + topic_);
      ti_ = ti;
      int gi = log_->ensure_group(ti, group_);
      GroupMeta& g = log_->h()->groups[gi];
      log_->reap(g, log_->h()->topics[ti].nparts);
      int slot = -1;
      for (int m = 0; m < kMaxMembers && slot < 0; ++m)
        if (!g.members[m].used) slot = m;
      if (slot < 0) throw std::runtime_error("shm log: too many members in group " + group_);
      copy_name(g.members[slot].id, member_, kMemberLen);
      g.members[slot].pid = (int32_t)getpid();
      g.members[slot].used = 1;
      g.nmembers++;
      log_->rebalance(g, log_->h()->topics[ti].nparts);
      slot_ = slot;
      gi_ = gi;
      gen_ = 0;
      started_ = true;
    }
    log_->notify();
  }

  void close() {
    py::gil_scoped_release nogil;
    if (!started_) return;
    {
      Locked l(log_->h());
      GroupMeta* g = group();
      if (g && g->members[slot_].used && member_ == g->members[slot_].id) {
        publish_locked(*g);
        g->members[slot_].used = 0;
        g->nmembers--;
        log_->rebalance(*g, log_->h()->topics[ti_].nparts);
      }
      started_ = false;
    }
    log_->notify();
  }

  std::vector<int> assignment() {
    py::gil_scoped_release nogil;
    Locked l(log_->h());
    std::vector<int> r;
    GroupMeta* g = group();
    if (!g) return r;
    for (int p = 0; p < log_->h()->topics[ti_].nparts; ++p)
      if (g->owner[p] == slot_) r.push_back(p);
    return r;
  }

  py::list poll(int max_records, double timeout_ms) {
    std::vector<Rec> recs;
    {
      py::gil_scoped_release nogil;
      const auto deadline =
          std::chrono::steady_clock::now() + std::chrono::microseconds((int64_t)(timeout_ms * 1000));
      while (started_) {
        const uint32_t s0 = log_->seq();
        {
          Locked l(log_->h());
          std::lock_guard<std::mutex> lk(mu_);
          GroupMeta* g = group();
          if (!g) break;
          const int np = log_->h()->topics[ti_].nparts;
          auto now = std::chrono::steady_clock::now();
          if (now - last_reap_ > std::chrono::milliseconds(500)) {
            last_reap_ = now;
            log_->reap(*g, np);
          }
          sync_assignment(*g, np);
          uint64_t budget = 16ull << 20;
          int n = 0;
          for (int k = 0; k < np && n < max_records && budget > 0; ++k) {
            const int p = (int)((rr_ + k) % np);
            if (!owned_[p]) continue;
            clamp_to_base(*g, p);
            n += log_->read_part(ti_, p, pos_[p], cur_[p], max_records - n, budget, recs);
          }
          rr_++;
        }
        if (!recs.empty() || !log_->wait_for(s0, deadline)) break;
      }
    }
    py::list out;
    for (auto& r : recs) out.append(py::make_tuple(r.part, r.off, py::bytes(r.data)));
    return out;
  }

  // Acknowledge offsets; the committed offset advances through the contiguous prefix
  // (KafkaConsumerWrapper.java:203-277) and is published when this member owns the
  // partition.  Returns the committed offsets of the touched partitions.
  std::map<int, int64_t> ack(const std::vector<std::pair<int, int64_t>>& offsets) {
    py::gil_scoped_release nogil;
    std::map<int, int64_t> res;
    Locked l(log_->h());
    std::lock_guard<std::mutex> lk(mu_);
    GroupMeta* g = group();
    if (!g) return res;
    const int np = log_->h()->topics[ti_].nparts;
    sync_assignment(*g, np);
    for (auto& po : offsets) {
      const int p = po.first;
      if (p < 0 || p >= np || !owned_[p]) continue;  // stale ack after a rebalance
      clamp_to_base(*g, p);
      if (po.second < committed_[p]) continue;
      done_[p].insert(po.second);
      while (!done_[p].empty() && *done_[p].begin() == committed_[p]) {
        done_[p].erase(done_[p].begin());
        committed_[p]++;
      }
      res[p] = committed_[p];
    }
    publish_locked(*g);
    return res;
  }

 private:
  GroupMeta* group() {
    if (gi_ < 0) return nullptr;
    GroupMeta& g = log_->h()->groups[gi_];
    if (!g.used || g.topic != ti_ || group_ != g.name) return nullptr;
    return &g;
  }

  // Retention dropped the head of partition p past offsets this group never committed
  // (a lagging consumer): those offsets can no longer be delivered or acked, so the
  // contiguous-prefix commit would freeze below them forever.  Move the committed offset
  // (ours and the group's published one) and the read position up to the partition's
  // first stored offset, and forget acks below it -- Kafka's "offset out of range ->
  // earliest" for a consumer overtaken by retention.
  void clamp_to_base(GroupMeta& g, int p) {
    const int64_t base = log_->part_base(ti_, p);
    if (committed_[p] < base) {
      committed_[p] = base;
      done_[p].erase(done_[p].begin(), done_[p].lower_bound(base));
      while (!done_[p].empty() && *done_[p].begin() == committed_[p]) {
        done_[p].erase(done_[p].begin());
        committed_[p]++;
      }
    }
    if (g.owner[p] == slot_ && g.committed[p] < committed_[p]) g.committed[p] = committed_[p];
    if (pos_[p] < base) {
      pos_[p] = base;
      cur_[p] = ShmLog::Cursor();
    }
  }

  void sync_assignment(GroupMeta& g, int np) {
    if (g.generation == gen_) return;
    for (int p = 0; p < np; ++p) {
      const bool mine = g.owner[p] == slot_;
      if (mine && (!owned_[p] || g.owner_since[p] > gen_)) {
        pos_[p] = g.committed[p];
        committed_[p] = g.committed[p];
        done_[p].clear();
        cur_[p] = ShmLog::Cursor();
      }
      if (!mine) done_[p].clear();
      owned_[p] = mine;
    }
    gen_ = g.generation;
  }

  void publish_locked(GroupMeta& g) {
    const int np = log_->h()->topics[ti_].nparts;
    for (int p = 0; p < np; ++p)
      if (owned_[p] && g.owner[p] == slot_ && committed_[p] > g.committed[p]) g.committed[p] = committed_[p];
  }

  std::shared_ptr<ShmLog> log_;
  std::string topic_, group_, member_;
  int ti_ = -1, gi_ = -1, slot_ = -1;
  bool started_ = false;
  uint64_t gen_ = 0;
  uint64_t rr_ = 0;
  std::mutex mu_;
  bool owned_[kMaxParts] = {};
  int64_t pos_[kMaxParts] = {};
  int64_t committed_[kMaxParts] = {};
  std::set<int64_t> done_[kMaxParts];
  ShmLog::Cursor cur_[kMaxParts];
  std::chrono::steady_clock::time_point last_reap_{};
};

// Group-less reader (gateways, tests): explicit per-partition positions.
class ShmReader {
 public:
  ShmReader(std::shared_ptr<ShmLog> log, std::string topic, std::vector<int64_t> positions)
      : log_(std::move(log)), topic_(std::move(topic)), pos_(std::move(positions)) {}

  py::list read(int max_records, double timeout_ms) {
    std::vector<Rec> recs;
    {
      py::gil_scoped_release nogil;
      const auto deadline =
          std::chrono::steady_clock::now() + std::chrono::microseconds((int64_t)(timeout_ms * 1000));
      while (true) {
        const uint32_t s0 = log_->seq();
        {
          Locked l(log_->h());
          std::lock_guard<std::mutex> lk(mu_);
          int ti = log_->find_topic(topic_);
          if (ti < 0) break;
          const int np = log_->h()->topics[ti].nparts;
          if ((int)pos_.size() < np) pos_.resize(np, 0);
          if ((int)cur_.size() < np) cur_.resize(np);
          uint64_t budget = 16ull << 20;
          int n = 0;
          for (int p = 0; p < np && n < max_records && budget > 0; ++p)
            n += log_->read_part(ti, p, pos_[p], cur_[p], max_records - n, budget, recs);
        }
        if (!recs.empty() || !log_->wait_for(s0, deadline)) break;
      }
    }
    py::list out;
    for (auto& r : recs) out.append(py::make_tuple(r.part, r.off, py::bytes(r.data)));
    return out;
  }

  std::vector<int64_t> positions() {
    std::lock_guard<std::mutex> lk(mu_);
    return pos_;
  }

 private:
  std::shared_ptr<ShmLog> log_;
  std::string topic_;
  std::vector<int64_t> pos_;
  std::vector<ShmLog::Cursor> cur_;
  std::mutex mu_;
};

}  // namespace

void bind_shmlog(py::module_& m) {
  py::class_<ShmLog, std::shared_ptr<ShmLog>>(m, "ShmLog")
      .def(py::init<const std::string&, uint64_t, uint64_t>(), py::arg("path"), py::arg("size"),
           py::arg("block_bytes") = 4u << 20, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("path", &ShmLog::path)
      .def_property_readonly("max_record", &ShmLog::max_record)
      .def("unlink", &ShmLog::unlink_file)
      .def("create_topic", &ShmLog::create_topic, py::arg("name"), py::arg("partitions") = 1,
           py::arg("retention") = 0, py::call_guard<py::gil_scoped_release>())
      .def("has_topic", &ShmLog::has_topic, py::call_guard<py::gil_scoped_release>())
      .def("delete_topic", &ShmLog::delete_topic, py::call_guard<py::gil_scoped_release>())
      .def("topics", &ShmLog::topics, py::call_guard<py::gil_scoped_release>())
      .def("partitions", &ShmLog::partitions, py::call_guard<py::gil_scoped_release>())
      .def(
          "append",
          [](ShmLog& self, const std::string& name, py::bytes data, int64_t key_hash, int partition,
             double timeout_ms) {
            std::string s = data;
            py::gil_scoped_release nogil;
            return self.append(name, s, key_hash, partition, timeout_ms);
          },
          py::arg("name"), py::arg("data"), py::arg("key_hash") = 0, py::arg("partition") = -1,
          py::arg("timeout_ms") = 30000.0)
      .def("end_offsets", &ShmLog::end_offsets, py::call_guard<py::gil_scoped_release>())
      .def("begin_offsets", &ShmLog::begin_offsets, py::call_guard<py::gil_scoped_release>())
      .def("total", &ShmLog::total, py::call_guard<py::gil_scoped_release>())
      .def("committed", &ShmLog::committed, py::call_guard<py::gil_scoped_release>())
      .def("lag", &ShmLog::lag, py::call_guard<py::gil_scoped_release>())
      .def("group_members", &ShmLog::group_members, py::call_guard<py::gil_scoped_release>())
      .def("groups", &ShmLog::groups, py::call_guard<py::gil_scoped_release>())
      .def("stats", &ShmLog::stats)
      .def("wakeup", &ShmLog::wakeup);
  py::class_<ShmConsumer, std::shared_ptr<ShmConsumer>>(m, "ShmConsumer")
      .def(py::init<std::shared_ptr<ShmLog>, std::string, std::string, std::string>())
      .def("start", &ShmConsumer::start)
      .def("close", &ShmConsumer::close)
      .def("assignment", &ShmConsumer::assignment)
      .def("poll", &ShmConsumer::poll, py::arg("max_records") = 500, py::arg("timeout_ms") = 200.0)
      .def("ack", &ShmConsumer::ack);
  py::class_<ShmReader, std::shared_ptr<ShmReader>>(m, "ShmReader")
      .def(py::init<std::shared_ptr<ShmLog>, std::string, std::vector<int64_t>>())
      .def("read", &ShmReader::read, py::arg("max_records") = 500, py::arg("timeout_ms") = 200.0)
      .def("positions", &ShmReader::positions);
  m.def("shmlog_close_gate", [] { g_closing.store(true); });
  m.def("shmlog_waiters", [] { return g_waiters.load(); });
}
