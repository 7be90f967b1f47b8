/* Host-only helpers of the checkpoint / summary writers (runtime/tf_bundle.py, runtime/metrics.py), built as
 * a plain CPython extension (_ina_host.so: no torch, no HIP), so CPU-only and evaluation hosts get them too.
 *
 * _ina_host.crc32c(buffer, crc=0): CRC-32C (Castagnoli) of any contiguous buffer (bytes, bytearray,
 * memoryview, a numpy array), continuing from `crc`.  TF's tensor bundle stores a masked CRC32C of every
 * tensor's bytes and of every SSTable block; the paper configuration's checkpoint (parameters + both Adam
 * moments) is ~86 MB, far too slow for a Python byte loop.  SSE4.2 crc32 instruction where the CPU has it,
 * slicing-by-8 tables otherwise.  The GIL is released while it runs. */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>
#include <string.h>

static uint32_t T[8][256];
static int T_ready = 0;

static void tables(void) {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
    T[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; ++i)
    for (int s = 1; s < 8; ++s) T[s][i] = (T[s - 1][i] >> 8) ^ T[0][T[s - 1][i] & 0xFF];
  T_ready = 1;
}

static uint32_t crc_sw(uint32_t c, const uint8_t* p, size_t n) {
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    v ^= c;
    c = T[7][v & 0xFF] ^ T[6][(v >> 8) & 0xFF] ^ T[5][(v >> 16) & 0xFF] ^ T[4][(v >> 24) & 0xFF] ^
        T[3][(v >> 32) & 0xFF] ^ T[2][(v >> 40) & 0xFF] ^ T[1][(v >> 48) & 0xFF] ^ T[0][v >> 56];
    p += 8;
    n -= 8;
  }
  while (n--) c = T[0][(c ^ *p++) & 0xFF] ^ (c >> 8);
  return c;
}

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) static uint32_t crc_hw(uint32_t c, const uint8_t* p, size_t n) {
  uint64_t c64 = c;
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    c64 = __builtin_ia32_crc32di(c64, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c64;
  while (n--) c32 = __builtin_ia32_crc32qi(c32, *p++);
  return c32;
}
#endif

static PyObject* py_crc32c(PyObject* self, PyObject* args) {
  Py_buffer buf;
  unsigned long long crc = 0;
  (void)self;
  if (!PyArg_ParseTuple(args, "y*|K", &buf, &crc)) return NULL;
  uint32_t c = ~(uint32_t)crc;
  Py_BEGIN_ALLOW_THREADS
#if defined(__x86_64__)
  if (__builtin_cpu_supports("sse4.2"))
    c = crc_hw(c, (const uint8_t*)buf.buf, (size_t)buf.len);
  else
    c = crc_sw(c, (const uint8_t*)buf.buf, (size_t)buf.len);
#else
  c = crc_sw(c, (const uint8_t*)buf.buf, (size_t)buf.len);
#endif
  Py_END_ALLOW_THREADS
  PyBuffer_Release(&buf);
  return PyLong_FromUnsignedLong((unsigned long)(~c));
}

static PyMethodDef methods[] = {
    {"crc32c", py_crc32c, METH_VARARGS, "crc32c(buffer, crc=0) -> CRC-32C of the buffer, continuing from crc"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_ina_host", "host-only IO helpers", -1, methods};

PyMODINIT_FUNC PyInit__ina_host(void) {
  if (!T_ready) tables();
  return PyModule_Create(&module);
}
