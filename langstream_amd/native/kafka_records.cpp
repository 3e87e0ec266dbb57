// Kafka RecordBatch v2 records section: encode / decode.
//
// Each record is varint(length) attributes varint(tsDelta) varint(offsetDelta)
// varint(keyLen) key varint(valueLen) value varint(#headers) {varint(kLen) k varint(vLen) v}
// with zigzag varints and -1 lengths for null.  The Python loops (topics/kafka/protocol.py
// _records / encode_batch) cost ~24 varint calls of ~2 us per record on every hop of a
// record (producer, consumer, reader) -- the per-record budget of the Kafka pipelines.
#include <Python.h>
#include <pybind11/pybind11.h>

#include <cstdint>
#include <stdexcept>
#include <string>

namespace py = pybind11;

namespace {

inline void put_varint(std::string& o, int64_t v) {
  uint64_t z = ((uint64_t)v << 1) ^ (uint64_t)(v >> 63);
  while (z >= 0x80) {
    o.push_back((char)((z & 0x7f) | 0x80));
    z >>= 7;
  }
  o.push_back((char)z);
}

inline int64_t get_varint(const uint8_t* b, size_t n, size_t& p) {
  uint64_t z = 0;
  int shift = 0;
  while (true) {
    if (p >= n || shift > 63) throw std::out_of_range("truncated Kafka record");
    uint8_t c = b[p++];
    z |= (uint64_t)(c & 0x7f) << shift;
    if (!(c & 0x80)) break;
    shift += 7;
  }
  return (int64_t)(z >> 1) ^ -(int64_t)(z & 1);
}

// bytes-like or None -> (ptr, len) with len = -1 for None
struct Blob {
  const char* p = nullptr;
  Py_ssize_t n = -1;
  Py_buffer view{};
  bool has_view = false;
  ~Blob() {
    if (has_view) PyBuffer_Release(&view);
  }
};

void get_blob(PyObject* o, Blob& b) {
  if (o == Py_None) return;
  if (PyBytes_Check(o)) {
    b.p = PyBytes_AS_STRING(o);
    b.n = PyBytes_GET_SIZE(o);
    return;
  }
  if (PyUnicode_Check(o)) {
    b.p = PyUnicode_AsUTF8AndSize(o, &b.n);
    if (!b.p) throw py::error_already_set();
    return;
  }
  if (PyObject_GetBuffer(o, &b.view, PyBUF_SIMPLE) != 0) throw py::error_already_set();
  b.has_view = true;
  b.p = (const char*)b.view.buf;
  b.n = b.view.len;
}

void put_blob(std::string& rec, PyObject* o) {
  Blob b;
  get_blob(o, b);
  put_varint(rec, b.n);
  if (b.n > 0) rec.append(b.p, b.n);
}

// records: sequence of (key, value, headers[(str, bytes|None)], timestamp_ms)
py::bytes encode_records(py::sequence records, int64_t first_ts) {
  std::string body, rec;
  body.reserve(256 * (size_t)py::len(records));
  Py_ssize_t i = 0;
  for (py::handle r : records) {
    py::tuple t = py::reinterpret_borrow<py::object>(r);
    if (t.size() != 4) throw std::invalid_argument("record must be (key, value, headers, timestamp)");
    rec.clear();
    rec.push_back('\0');
    put_varint(rec, t[3].cast<int64_t>() - first_ts);
    put_varint(rec, i);
    put_blob(rec, t[0].ptr());
    put_blob(rec, t[1].ptr());
    py::sequence hs = py::reinterpret_borrow<py::sequence>(t[2]);
    put_varint(rec, (int64_t)py::len(hs));
    for (py::handle h : hs) {
      py::tuple hv = py::reinterpret_borrow<py::object>(h);
      put_blob(rec, hv[0].ptr());
      put_blob(rec, hv[1].ptr());
    }
    put_varint(body, (int64_t)rec.size());
    body.append(rec);
    ++i;
  }
  return py::bytes(body);
}

PyObject* bytes_or_none(const uint8_t* b, int64_t len, size_t& p, size_t n) {
  if (len < 0) Py_RETURN_NONE;
  if (p + (size_t)len > n) throw std::out_of_range("truncated Kafka record");
  PyObject* o = PyBytes_FromStringAndSize((const char*)b + p, (Py_ssize_t)len);
  p += (size_t)len;
  if (!o) throw py::error_already_set();
  return o;
}

// -> [(offset, timestamp, key, value, [(header key str, header value)])]
py::list decode_records(py::buffer data, size_t p, int64_t count, int64_t base, int64_t first_ts) {
  py::buffer_info bi = data.request();
  const uint8_t* b = (const uint8_t*)bi.ptr;
  const size_t n = (size_t)bi.size * (size_t)bi.itemsize;
  py::list out;
  for (int64_t i = 0; i < count; ++i) {
    get_varint(b, n, p);   // record length
    p += 1;                // attributes
    int64_t tsd = get_varint(b, n, p);
    int64_t od = get_varint(b, n, p);
    py::object key = py::reinterpret_steal<py::object>(bytes_or_none(b, get_varint(b, n, p), p, n));
    py::object val = py::reinterpret_steal<py::object>(bytes_or_none(b, get_varint(b, n, p), p, n));
    int64_t nh = get_varint(b, n, p);
    py::list hs;
    for (int64_t h = 0; h < nh; ++h) {
      int64_t kl = get_varint(b, n, p);
      if (kl < 0 || p + (size_t)kl > n) throw std::out_of_range("truncated Kafka record header");
      PyObject* hk = PyUnicode_DecodeUTF8((const char*)b + p, (Py_ssize_t)kl, nullptr);
      if (!hk) throw py::error_already_set();
      p += (size_t)kl;
      py::object hko = py::reinterpret_steal<py::object>(hk);
      py::object hvo = py::reinterpret_steal<py::object>(bytes_or_none(b, get_varint(b, n, p), p, n));
      hs.append(py::make_tuple(hko, hvo));
    }
    out.append(py::make_tuple(base + od, first_ts + tsd, key, val, hs));
  }
  return out;
}

}  // namespace

void bind_kafka_records(py::module_& m) {
  m.def("kafka_encode_records", &encode_records, py::arg("records"), py::arg("first_ts"),
        "RecordBatch v2 records section of (key, value, headers, ts) tuples");
  m.def("kafka_decode_records", &decode_records, py::arg("data"), py::arg("pos"), py::arg("count"),
        py::arg("base_offset"), py::arg("first_ts"),
        "records of one uncompressed records section -> [(offset, ts, key, value, headers)]");
}
