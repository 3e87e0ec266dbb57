// json_dumps(obj) -> str: the text the reference runtime puts on a topic for a map /
// list value (Jackson's ObjectMapper.writeValueAsString: compact "," / ":" separators,
// non-ASCII characters written as themselves, control characters escaped), which is
// byte-identical to Python's json.dumps(obj, separators=(",", ":"), ensure_ascii=False)
// (allow_nan, insertion-ordered keys) for dict / list / tuple / str / int / float /
// bool / None trees.  Numbers keep Python's repr digits.
//
// Why native: records leaving an embeddings agent carry a 384..1024-float vector, and
// json.dumps spends ~0.7 us per float in float.__repr__ + str building (263 us for one
// bge-small record, measured) -- the whole per-record budget of the Kafka embeddings
// pipeline (BASELINE config 2).  Floats here go through std::to_chars (shortest
// round-trip digits, the digits repr() picks) laid out by repr's rules: positional for
// decimal exponents -4..15 with a ".0" for integral values, else d.ddde+XX.
//
// Anything else (numpy scalars, objects with a `default`, cycles deeper than the
// limit, strings with lone surrogates) raises _lsnative.JsonUnsupported and the Python
// wrapper falls back to json.dumps with the same options, so errors and extensions
// behave exactly as before.
//
// Float32 vectors: a list of the registered float32-vector type (utils/fastjson.py
// Float32List: the embeddings of a local float32 / bf16 model) is written with each
// value's shortest float32 round-trip digits (to_chars(float)), in repr's layout --
// exactly what json.dumps prints for the doubles those digits parse to.  A float32
// value widened to a double has ~17 significant digits; the float32 digits are ~9, so
// the record is half the bytes and the formatting ~4x cheaper, with no information
// lost (float32(parsed value) is the original float32).
#include <Python.h>
#include <pybind11/pybind11.h>
#include <pybind11/numpy.h>

#include <charconv>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace py = pybind11;

namespace {

PyObject* g_unsupported = nullptr;
PyTypeObject* g_f32list = nullptr;   // utils.fastjson.Float32List, registered at import

struct Unsupported {};

const char HEX[] = "0123456789abcdef";

void put_u16(std::string& o, unsigned c) {
  char b[6] = {'\\', 'u', HEX[(c >> 12) & 15], HEX[(c >> 8) & 15], HEX[(c >> 4) & 15], HEX[c & 15]};
  o.append(b, 6);
}

inline void put_utf8(std::string& o, Py_UCS4 c) {
  if (c < 0x80) {
    o.push_back((char)c);
  } else if (c < 0x800) {
    o.push_back((char)(0xc0 | (c >> 6)));
    o.push_back((char)(0x80 | (c & 0x3f)));
  } else if (c < 0x10000) {
    if (c >= 0xd800 && c <= 0xdfff) throw Unsupported{};   // lone surrogate: json's own path
    o.push_back((char)(0xe0 | (c >> 12)));
    o.push_back((char)(0x80 | ((c >> 6) & 0x3f)));
    o.push_back((char)(0x80 | (c & 0x3f)));
  } else {
    o.push_back((char)(0xf0 | (c >> 18)));
    o.push_back((char)(0x80 | ((c >> 12) & 0x3f)));
    o.push_back((char)(0x80 | ((c >> 6) & 0x3f)));
    o.push_back((char)(0x80 | (c & 0x3f)));
  }
}

inline bool put_escape(std::string& o, Py_UCS4 c) {
  switch (c) {
    case '"': o.append("\\\""); return true;
    case '\\': o.append("\\\\"); return true;
    case '\n': o.append("\\n"); return true;
    case '\r': o.append("\\r"); return true;
    case '\t': o.append("\\t"); return true;
    case '\b': o.append("\\b"); return true;
    case '\f': o.append("\\f"); return true;
    default:
      if (c < 0x20) { put_u16(o, c); return true; }
      return false;
  }
}

void put_str(std::string& o, PyObject* s) {
  if (PyUnicode_READY(s) < 0) throw Unsupported{};
  const Py_ssize_t n = PyUnicode_GET_LENGTH(s);
  const int kind = PyUnicode_KIND(s);
  const void* d = PyUnicode_DATA(s);
  o.push_back('"');
  if (PyUnicode_IS_ASCII(s)) {
    const unsigned char* p = (const unsigned char*)d;
    Py_ssize_t i = 0;
    while (i < n) {
      // copy the run of characters that need no escape in one append
      Py_ssize_t j = i;
      while (j < n && p[j] >= 0x20 && p[j] != '"' && p[j] != '\\') ++j;
      if (j > i) o.append((const char*)p + i, j - i);
      if (j >= n) break;
      put_escape(o, p[j]);
      i = j + 1;
    }
  } else {
    for (Py_ssize_t i = 0; i < n; ++i) {
      const Py_UCS4 c = PyUnicode_READ(kind, d, i);
      if (!put_escape(o, c)) put_utf8(o, c);
    }
  }
  o.push_back('"');
}

// float.__repr__ layout over the shortest round-trip digits, built in one stack buffer
// (appending piecewise to the std::string cost as much as the digit generation)
template <typename T>
inline int format_float(char* out, T x) {
  char* w = out;
  if (std::isnan(x)) { std::memcpy(w, "NaN", 3); return 3; }
  if (std::isinf(x)) {
    if (x > 0) { std::memcpy(w, "Infinity", 8); return 8; }
    std::memcpy(w, "-Infinity", 9); return 9;
  }
  if (x == 0) {
    if (std::signbit(x)) { std::memcpy(w, "-0.0", 4); return 4; }
    std::memcpy(w, "0.0", 3); return 3;
  }
  char buf[40];
  auto r = std::to_chars(buf, buf + sizeof buf, x, std::chars_format::scientific);
  if (r.ec != std::errc()) throw Unsupported{};
  // buf = [-]d[.ddd]e(+|-)XX
  const char* p = buf;
  const char* end = r.ptr;
  if (*p == '-') { *w++ = '-'; ++p; }
  char dig[24];
  int nd = 0;
  dig[nd++] = *p++;
  if (*p == '.') {
    ++p;
    while (*p != 'e') dig[nd++] = *p++;
  }
  // exponent: e, sign, 2..3 digits
  const bool eneg = p[1] == '-';
  int e = 0;
  for (const char* q = p + 2; q < end; ++q) e = e * 10 + (*q - '0');
  if (eneg) e = -e;
  if (e >= -4 && e < 16) {
    if (e < 0) {
      *w++ = '0'; *w++ = '.';
      for (int i = 0; i < -e - 1; ++i) *w++ = '0';
      std::memcpy(w, dig, nd); w += nd;
    } else if (nd <= e + 1) {
      std::memcpy(w, dig, nd); w += nd;
      for (int i = 0; i < e + 1 - nd; ++i) *w++ = '0';
      *w++ = '.'; *w++ = '0';
    } else {
      std::memcpy(w, dig, e + 1); w += e + 1;
      *w++ = '.';
      std::memcpy(w, dig + e + 1, nd - e - 1); w += nd - e - 1;
    }
  } else {
    *w++ = dig[0];
    if (nd > 1) {
      *w++ = '.';
      std::memcpy(w, dig + 1, nd - 1); w += nd - 1;
    }
    *w++ = 'e';
    *w++ = e < 0 ? '-' : '+';
    int a = e < 0 ? -e : e;
    if (a >= 100) { *w++ = char('0' + a / 100); a %= 100; *w++ = char('0' + a / 10); *w++ = char('0' + a % 10); }
    else { *w++ = char('0' + a / 10); *w++ = char('0' + a % 10); }
  }
  return int(w - out);
}

void put_float(std::string& o, double x) {
  char b[48];
  o.append(b, format_float(b, x));
}

// a Float32List: every item a float (anything else: the generic path)
bool put_f32_list(std::string& o, PyObject* seq) {
  const Py_ssize_t n = PyList_GET_SIZE(seq);
  // Float32List is a mutable list: user or EL code may have stored doubles in it.  Only
  // when every item is exactly a float32 value are float32 shortest digits the same
  // number; otherwise the generic path writes doubles (json.dumps' digits).
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* it = PyList_GET_ITEM(seq, i);
    if (!PyFloat_CheckExact(it)) return false;
    const double d = PyFloat_AS_DOUBLE(it);
    if ((double)(float)d != d && d == d) return false;
  }
  const size_t at = o.size();
  o.resize(at + size_t(n) * 24 + 2);   // "," + at most 18 chars per float32, + brackets
  char* w = &o[at];
  char* const w0 = w;
  *w++ = '[';
  for (Py_ssize_t i = 0; i < n; ++i) {
    if (i) *w++ = ',';
    w += format_float(w, (float)PyFloat_AS_DOUBLE(PyList_GET_ITEM(seq, i)));
  }
  *w++ = ']';
  o.resize(at + size_t(w - w0));
  return true;
}

void put_int(std::string& o, PyObject* v) {
  int overflow = 0;
  long long x = PyLong_AsLongLongAndOverflow(v, &overflow);
  if (overflow == 0) {
    if (x == -1 && PyErr_Occurred()) { PyErr_Clear(); throw Unsupported{}; }
    char b[24];
    auto r = std::to_chars(b, b + sizeof b, x);
    o.append(b, r.ptr - b);
    return;
  }
  PyObject* s = PyObject_Str(v);   // int.__str__ is int.__repr__
  if (!s) { PyErr_Clear(); throw Unsupported{}; }
  Py_ssize_t n;
  const char* c = PyUnicode_AsUTF8AndSize(s, &n);
  if (c) o.append(c, n);
  Py_DECREF(s);
  if (!c) { PyErr_Clear(); throw Unsupported{}; }
}

void put(std::string& o, PyObject* v, int depth);

// LS_JSON_NOGIL=1: a long all-float list (an embedding vector) is formatted with the GIL
// released (the doubles are copied out first; the list is never touched without the
// GIL).  Off by default: measured on the config-2 agent (bench/embed.py, null embedder)
// it LOST 20-30% -- the releasing thread then waits a switch interval to get the GIL
// back from the agent's CPU-bound threads, which costs more than the ~25 us/record of
// formatting it overlaps.
constexpr Py_ssize_t kFloatRunMin = 64;

bool float_run_enabled() {
  static const bool on = [] {
    const char* e = getenv("LS_JSON_NOGIL");
    return e != nullptr && e[0] == '1';
  }();
  return on;
}

bool put_float_run(std::string& o, PyObject* seq, bool lst, Py_ssize_t n) {
  thread_local std::vector<double> xs;
  thread_local std::string tmp;
  xs.resize(n);
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* it = lst ? PyList_GET_ITEM(seq, i) : PyTuple_GET_ITEM(seq, i);
    if (!PyFloat_CheckExact(it)) return false;
    xs[i] = PyFloat_AS_DOUBLE(it);
  }
  // "," + at most 25 chars per float, + brackets
  tmp.resize(size_t(n) * 28 + 2);
  size_t len = 0;
  bool ok = true;
  Py_BEGIN_ALLOW_THREADS
  try {
    char* w = &tmp[0];
    *w++ = '[';
    for (Py_ssize_t i = 0; i < n; ++i) {
      if (i) *w++ = ',';
      w += format_float(w, xs[i]);
    }
    *w++ = ']';
    len = size_t(w - &tmp[0]);
  } catch (...) {
    ok = false;
  }
  Py_END_ALLOW_THREADS
  if (!ok) throw Unsupported{};
  o.append(tmp.data(), len);
  return true;
}

void put_key(std::string& o, PyObject* k) {
  if (PyUnicode_Check(k)) { put_str(o, k); return; }
  // json.dumps coerces these key types to strings
  o.push_back('"');
  if (k == Py_True) o.append("true");
  else if (k == Py_False) o.append("false");
  else if (k == Py_None) o.append("null");
  else if (PyFloat_Check(k)) put_float(o, PyFloat_AS_DOUBLE(k));
  else if (PyLong_Check(k)) put_int(o, k);
  else throw Unsupported{};
  o.push_back('"');
}

void put(std::string& o, PyObject* v, int depth) {
  if (depth > 200) throw Unsupported{};   // let json.dumps report recursion / cycles
  if (PyUnicode_Check(v)) { put_str(o, v); return; }
  if (v == Py_None) { o.append("null"); return; }
  if (v == Py_True) { o.append("true"); return; }
  if (v == Py_False) { o.append("false"); return; }
  if (PyFloat_Check(v)) {
    // a float subclass with its own __repr__ would differ; json.dumps uses float.__repr__
    put_float(o, PyFloat_AS_DOUBLE(v));
    return;
  }
  if (PyLong_Check(v)) {
    if (!PyLong_CheckExact(v)) throw Unsupported{};   // IntEnum etc.: json's own rules
    put_int(o, v);
    return;
  }
  if (g_f32list != nullptr && Py_TYPE(v) == g_f32list && put_f32_list(o, v)) return;
  if (PyList_Check(v) || PyTuple_Check(v)) {
    PyObject* seq = v;
    const bool lst = PyList_Check(v);
    Py_ssize_t n = lst ? PyList_GET_SIZE(seq) : PyTuple_GET_SIZE(seq);
    if (n >= kFloatRunMin && float_run_enabled() && put_float_run(o, seq, lst, n)) return;
    o.push_back('[');
    for (Py_ssize_t i = 0; i < n; ++i) {
      if (i) o.push_back(',');
      PyObject* it = lst ? PyList_GET_ITEM(seq, i) : PyTuple_GET_ITEM(seq, i);
      Py_INCREF(it);
      try {
        put(o, it, depth + 1);
      } catch (...) {
        Py_DECREF(it);
        throw;
      }
      Py_DECREF(it);
      if (lst) n = PyList_GET_SIZE(seq);
    }
    o.push_back(']');
    return;
  }
  if (PyDict_Check(v)) {
    if (!PyDict_CheckExact(v)) throw Unsupported{};   // OrderedDict & co: json's own path
    o.push_back('{');
    Py_ssize_t pos = 0;
    PyObject *k, *x;
    bool first = true;
    while (PyDict_Next(v, &pos, &k, &x)) {
      if (!first) o.push_back(',');
      first = false;
      put_key(o, k);
      o.push_back(':');
      Py_INCREF(x);
      try {
        put(o, x, depth + 1);
      } catch (...) {
        Py_DECREF(x);
        throw;
      }
      Py_DECREF(x);
    }
    o.push_back('}');
    return;
  }
  throw Unsupported{};
}

py::object json_dumps(py::handle obj) {
  std::string o;
  o.reserve(256);
  try {
    put(o, obj.ptr(), 0);
  } catch (const Unsupported&) {
    PyErr_SetString(g_unsupported, "json_dumps: type outside the native encoder");
    throw py::error_already_set();
  }
  // output is UTF-8
  PyObject* s = PyUnicode_FromStringAndSize(o.data(), (Py_ssize_t)o.size());
  if (!s) throw py::error_already_set();
  return py::reinterpret_steal<py::object>(s);
}

}  // namespace

void bind_jsonenc(py::module_& m) {
  g_unsupported = PyErr_NewException("_lsnative.JsonUnsupported", PyExc_TypeError, nullptr);
  m.attr("JsonUnsupported") = py::handle(g_unsupported);
  m.def("json_dumps", &json_dumps, py::arg("obj"),
        "json.dumps(obj, separators=(',', ':'), ensure_ascii=False); raises JsonUnsupported for other types");
  // rows of a C-contiguous float32 [n, d] buffer -> n Float32Lists (the embedding engine's
  // results): the PyFloats are made here, ~10x cheaper than ndarray.tolist() + a copy
  m.def("f32_rows", [](py::buffer b) {
    if (g_f32list == nullptr) throw py::value_error("json_register_f32list first");
    py::buffer_info bi = b.request();
    if (bi.format != py::format_descriptor<float>::format() || bi.ndim != 2 ||
        bi.strides[1] != (py::ssize_t)sizeof(float) || bi.strides[0] != bi.shape[1] * (py::ssize_t)sizeof(float))
      throw py::value_error("f32_rows: a C-contiguous float32 [n, d] buffer");
    const py::ssize_t n = bi.shape[0], d = bi.shape[1];
    const float* x = static_cast<const float*>(bi.ptr);
    py::list out(n);
    for (py::ssize_t i = 0; i < n; ++i) {
      PyObject* plain = PyList_New(d);
      if (!plain) throw py::error_already_set();
      for (py::ssize_t j = 0; j < d; ++j) {
        PyObject* f = PyFloat_FromDouble((double)x[i * d + j]);
        if (!f) { Py_DECREF(plain); throw py::error_already_set(); }
        PyList_SET_ITEM(plain, j, f);
      }
      PyObject* row = PyObject_CallOneArg(reinterpret_cast<PyObject*>(g_f32list), plain);
      Py_DECREF(plain);
      if (!row) throw py::error_already_set();
      PyList_SET_ITEM(out.ptr(), i, row);
    }
    return out;
  }, py::arg("rows"));
  // the inverse: a sequence of equal-length number lists (e.g. the retrieved documents'
  // Float32List vectors the re-rank agent scores) -> a float32 [n, d] array, reading the
  // PyFloats directly (np.asarray over Python floats cost ~0.2 ms for 20 x 384)
  m.def("f32_matrix", [](py::sequence rows) {
    const py::ssize_t n = (py::ssize_t)py::len(rows);
    py::ssize_t d = -1;
    std::vector<float> buf;
    for (py::ssize_t i = 0; i < n; ++i) {
      PyObject* r = PySequence_GetItem(rows.ptr(), i);
      if (!r) throw py::error_already_set();
      PyObject* fast = PySequence_Fast(r, "f32_matrix: rows must be sequences");
      Py_DECREF(r);
      if (!fast) throw py::error_already_set();
      const py::ssize_t m = PySequence_Fast_GET_SIZE(fast);
      if (d < 0) { d = m; buf.reserve((size_t)(n * d)); }
      if (m != d) { Py_DECREF(fast); throw py::value_error("f32_matrix: ragged rows"); }
      PyObject** items = PySequence_Fast_ITEMS(fast);
      for (py::ssize_t j = 0; j < m; ++j) {
        PyObject* o = items[j];
        double v;
        if (PyFloat_CheckExact(o)) v = PyFloat_AS_DOUBLE(o);
        else {
          if (PyBool_Check(o) || !PyNumber_Check(o)) { Py_DECREF(fast); throw py::value_error("f32_matrix: non-numeric entry"); }
          v = PyFloat_AsDouble(o);
          if (v == -1.0 && PyErr_Occurred()) { Py_DECREF(fast); throw py::error_already_set(); }
        }
        buf.push_back((float)v);
      }
      Py_DECREF(fast);
    }
    if (d < 0) d = 0;
    py::array_t<float> out({n, d});
    if (n * d) std::memcpy(out.mutable_data(), buf.data(), sizeof(float) * (size_t)(n * d));
    return out;
  }, py::arg("rows"));
  m.def("json_register_f32list", [](py::handle t) {
    if (!PyType_Check(t.ptr())) throw py::type_error("a type");
    Py_INCREF(t.ptr());
    g_f32list = reinterpret_cast<PyTypeObject*>(t.ptr());
  }, "register the list subclass whose float items are float32 values");
}
