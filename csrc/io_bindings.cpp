// Host-side IO helpers of the checkpoint / summary writers (runtime/tf_bundle.py, runtime/metrics.py).
//
// ina.crc32c(data, crc): CRC-32C (Castagnoli) of a contiguous CPU byte tensor, continuing from `crc`
// (0 to start).  TF's tensor bundle stores a masked CRC32C of every tensor's bytes and of every SSTable
// block; the paper configuration's checkpoint is ~86 MB, far too slow for a Python byte loop.  Uses the
// SSE4.2 crc32 instruction (three interleaved streams would be faster still; one stream is ~8 GB/s,
// plenty here) with a slicing-by-8 table fallback on CPUs without it.
#include <ATen/ATen.h>
#include <torch/library.h>

#include <cstdint>
#include <cstring>

namespace {

struct Tables {
  uint32_t t[8][256];
  Tables() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFF];
  }
};

uint32_t crc_sw(uint32_t c, const uint8_t* p, size_t n) {
  static const Tables T;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    v ^= c;
    c = T.t[7][v & 0xFF] ^ T.t[6][(v >> 8) & 0xFF] ^ T.t[5][(v >> 16) & 0xFF] ^ T.t[4][(v >> 24) & 0xFF] ^
        T.t[3][(v >> 32) & 0xFF] ^ T.t[2][(v >> 40) & 0xFF] ^ T.t[1][(v >> 48) & 0xFF] ^ T.t[0][v >> 56];
    p += 8;
    n -= 8;
  }
  while (n--) c = T.t[0][(c ^ *p++) & 0xFF] ^ (c >> 8);
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
#endif

int64_t crc32c(const at::Tensor& data, int64_t crc) {
  TORCH_CHECK(!data.is_cuda() && data.is_contiguous() && data.scalar_type() == at::kByte,
              "ina.crc32c: data must be a contiguous CPU uint8 tensor");
  const uint8_t* p = data.data_ptr<uint8_t>();
  const size_t n = (size_t)data.numel();
  uint32_t c = ~(uint32_t)crc;
#if defined(__x86_64__)
  static const bool hw = __builtin_cpu_supports("sse4.2");
  c = hw ? crc_hw(c, p, n) : crc_sw(c, p, n);
#else
  c = crc_sw(c, p, n);
#endif
  return (int64_t)(~c);
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(ina, m) { m.def("crc32c", &crc32c); }
