// Checksums of the Kafka wire protocol, native: CRC-32C (Castagnoli) of every record
// batch (v2 record batches carry it; the producer computes it, the broker and the
// consumer verify it) and the murmur2 hash of the default partitioner.  A pure-Python
// byte loop ran CRC-32C at a few MB/s, which capped an embeddings agent writing ~8 KB
// JSON vectors per record at a few hundred records/s (BASELINE config 2).
//
// CRC-32C uses the SSE4.2 crc32 instruction (8 bytes per instruction) when the CPU has
// it, else a slice-by-8 table; the GIL is released only for very large buffers.
#include <pybind11/pybind11.h>

#include <cstdint>
#include <cstring>

namespace py = pybind11;

namespace {

uint32_t g_tab[8][256];

void init_tables() {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
    g_tab[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; ++i)
    for (int s = 1; s < 8; ++s) g_tab[s][i] = (g_tab[s - 1][i] >> 8) ^ g_tab[0][g_tab[s - 1][i] & 0xFF];
}

uint32_t crc_table(uint32_t c, const uint8_t* p, size_t n) {
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    v ^= c;
    c = g_tab[7][v & 0xFF] ^ g_tab[6][(v >> 8) & 0xFF] ^ g_tab[5][(v >> 16) & 0xFF] ^ g_tab[4][(v >> 24) & 0xFF] ^
        g_tab[3][(v >> 32) & 0xFF] ^ g_tab[2][(v >> 40) & 0xFF] ^ g_tab[1][(v >> 48) & 0xFF] ^ g_tab[0][v >> 56];
    p += 8;
    n -= 8;
  }
  while (n--) c = g_tab[0][(c ^ *p++) & 0xFF] ^ (c >> 8);
  return c;
}

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) uint32_t crc_hw(uint32_t c, const uint8_t* p, size_t n) {
  uint64_t c64 = c;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    c64 = __builtin_ia32_crc32di(c64, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c64;
  while (n--) c32 = __builtin_ia32_crc32qi(c32, *p++);
  return c32;
}
bool have_hw() {
  static const bool v = __builtin_cpu_supports("sse4.2");
  return v;
}
#else
uint32_t crc_hw(uint32_t c, const uint8_t* p, size_t n) { return crc_table(c, p, n); }
bool have_hw() { return false; }
#endif

uint32_t crc32c(uint32_t crc, const uint8_t* p, size_t n) {
  const uint32_t c = ~crc;
  return ~(have_hw() ? crc_hw(c, p, n) : crc_table(c, p, n));
}

uint32_t crc32c_py(py::buffer b, uint32_t crc) {
  py::buffer_info info = b.request();
  const auto* p = static_cast<const uint8_t*>(info.ptr);
  const size_t n = (size_t)(info.size * info.itemsize);
  // release the GIL only for work well above a switch interval's worth: re-taking a
  // contended GIL costs up to the 5 ms switch interval, ~40 MB of CRC at 8 GB/s
  if (n >= (1 << 23)) {
    py::gil_scoped_release rel;
    return crc32c(crc, p, n);
  }
  return crc32c(crc, p, n);
}

// Kafka's murmur2 (the Java client's Utils.murmur2): seed 0x9747b28c, 4-byte little-endian words.
int32_t murmur2(py::bytes data) {
  std::string s = data;
  const auto* d = reinterpret_cast<const uint8_t*>(s.data());
  const int len = (int)s.size();
  const uint32_t m = 0x5bd1e995u;
  const int r = 24;
  uint32_t h = 0x9747b28cu ^ (uint32_t)len;
  const int n4 = len / 4;
  for (int i = 0; i < n4; ++i) {
    uint32_t k = (uint32_t)d[4 * i] | ((uint32_t)d[4 * i + 1] << 8) | ((uint32_t)d[4 * i + 2] << 16) |
                 ((uint32_t)d[4 * i + 3] << 24);
    k *= m;
    k ^= k >> r;
    k *= m;
    h *= m;
    h ^= k;
  }
  const int t = len & 3, o = len & ~3;
  if (t == 3) h ^= (uint32_t)d[o + 2] << 16;
  if (t >= 2) h ^= (uint32_t)d[o + 1] << 8;
  if (t >= 1) {
    h ^= (uint32_t)d[o];
    h *= m;
  }
  h ^= h >> 13;
  h *= m;
  h ^= h >> 15;
  return (int32_t)h;
}

}  // namespace

void bind_codec(py::module_& m) {
  init_tables();
  m.def("crc32c", &crc32c_py, py::arg("data"), py::arg("crc") = 0u,
        "CRC-32C (Castagnoli) of a bytes-like object, continuing from `crc`");
  m.def("crc32c_hw", [] { return have_hw(); });
  m.def("murmur2", &murmur2, "Kafka murmur2 hash (signed 32-bit, as the Java client)");
}
