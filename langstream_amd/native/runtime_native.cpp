// Native runtime pieces for the GPU engines + the module definition of _lsnative.
//
//  * BlockAllocator: paged-KV block manager (free list + reference counts so prefix
//    blocks can be shared between sequences).  O(1) alloc/free, used by the LLM engine
//    scheduler on every step.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <stdexcept>
#include <vector>

namespace py = pybind11;

void bind_memlog(py::module_& m);
void bind_shmlog(py::module_& m);
void bind_tokenizer(py::module_& m);
void bind_codec(py::module_& m);
void bind_jsonenc(py::module_& m);
void bind_kafka_records(py::module_& m);

namespace {

class BlockAllocator {
 public:
  explicit BlockAllocator(int num_blocks) : ref_(num_blocks, 0) {
    free_.reserve(num_blocks);
    for (int i = num_blocks - 1; i >= 0; --i) free_.push_back(i);
  }
  int num_free() const { return (int)free_.size(); }
  int num_blocks() const { return (int)ref_.size(); }
  bool can_allocate(int n) const { return n <= (int)free_.size(); }
  std::vector<int> allocate(int n) {
    if (n > (int)free_.size()) throw std::runtime_error("out of KV blocks");
    std::vector<int> r(n);
    for (int i = 0; i < n; ++i) {
      r[i] = free_.back();
      free_.pop_back();
      ref_[r[i]] = 1;
    }
    return r;
  }
  void incref(const std::vector<int>& blocks) {
    for (int b : blocks) check(b), ref_[b]++;
  }
  void free(const std::vector<int>& blocks) {
    for (int b : blocks) {
      check(b);
      if (ref_[b] <= 0) throw std::runtime_error("double free of KV block");
      if (--ref_[b] == 0) free_.push_back(b);
    }
  }
  int refcount(int b) const { check(b); return ref_[b]; }

 private:
  void check(int b) const {
    if (b < 0 || b >= (int)ref_.size()) throw std::out_of_range("bad KV block id");
  }
  std::vector<int> free_;
  std::vector<int> ref_;
};

}  // namespace

PYBIND11_MODULE(_lsnative, m) {
  m.doc() = "langstream_amd native host runtime (memlog, shared-memory log, tokenizers, KV block allocator, Kafka checksums, JSON encoder)";
  py::class_<BlockAllocator>(m, "BlockAllocator")
      .def(py::init<int>())
      .def("num_free", &BlockAllocator::num_free)
      .def("num_blocks", &BlockAllocator::num_blocks)
      .def("can_allocate", &BlockAllocator::can_allocate)
      .def("allocate", &BlockAllocator::allocate)
      .def("incref", &BlockAllocator::incref)
      .def("free", &BlockAllocator::free)
      .def("refcount", &BlockAllocator::refcount);
  bind_memlog(m);
  bind_shmlog(m);
  bind_tokenizer(m);
  bind_codec(m);
  bind_jsonenc(m);
  bind_kafka_records(m);
}
