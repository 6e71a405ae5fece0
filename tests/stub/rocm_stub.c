/* rocm_stub.c — a CPU stand-in for the few libamdhip64 / librccl entry points
 * sparc_ldpc_amd/dist.py:RcclComm binds, so its world > 1 bootstrap and
 * all-reduce sequence can run on a machine without GPUs
 * (tests/test_dist_stub.py).  Test infrastructure only: never shipped, never
 * loaded by the product.
 *
 * Every call appends one line to the file named by $STUB_LOG.  The unique id
 * is a fixed 128-byte pattern full of NUL bytes (the case a C-string read
 * truncates); ncclCommInitRank logs the id it received in hex.  ncclAllReduce
 * really reduces across the processes of a test: rank r writes its send
 * buffer to $STUB_DIR/ar_<call>_<r>.bin (write + rename), waits for every
 * rank's file of the same call and reduces them in rank order.
 */
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

typedef struct { char internal[128]; } ncclUniqueId;

static int g_rank = -1, g_world = 0, g_calls = 0;

static void logf_(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
static void logf_(const char* fmt, ...) {
  const char* p = getenv("STUB_LOG");
  if (!p) return;
  FILE* f = fopen(p, "a");
  if (!f) return;
  va_list ap;
  va_start(ap, fmt);
  vfprintf(f, fmt, ap);
  va_end(ap);
  fputc('\n', f);
  fclose(f);
}

static unsigned char pattern_byte(int i) { return (i % 3 == 2) ? 0 : (unsigned char)((i * 7 + 1) & 0xff); }

/* ---- libamdhip64 ---- */
int hipSetDevice(int d) { logf_("hipSetDevice %d", d); return 0; }
int hipStreamCreate(void** s) { *s = (void*)(uintptr_t)0x5100; logf_("hipStreamCreate"); return 0; }
int hipMalloc(void** p, size_t n) { *p = malloc(n); logf_("hipMalloc %zu", n); return *p ? 0 : 2; }
int hipFree(void* p) { free(p); logf_("hipFree"); return 0; }
int hipStreamDestroy(void* s) { (void)s; logf_("hipStreamDestroy"); return 0; }
int hipStreamSynchronize(void* s) { (void)s; logf_("hipStreamSynchronize"); return 0; }
int hipMemcpyAsync(void* dst, const void* src, size_t n, int kind, void* s) {
  (void)s;
  memcpy(dst, src, n);
  logf_("hipMemcpyAsync %zu %d", n, kind);
  return 0;
}

/* ---- librccl ---- */
const char* ncclGetErrorString(int rc) { (void)rc; return "stub error"; }

int ncclGetUniqueId(ncclUniqueId* id) {
  for (int i = 0; i < 128; ++i) id->internal[i] = (char)pattern_byte(i);
  logf_("ncclGetUniqueId");
  return 0;
}

int ncclCommInitRank(void** comm, int nranks, ncclUniqueId id, int rank) {
  char hex[257];
  for (int i = 0; i < 128; ++i) sprintf(hex + 2 * i, "%02x", (unsigned char)id.internal[i]);
  int ok = 1;
  for (int i = 0; i < 128; ++i) ok &= (unsigned char)id.internal[i] == pattern_byte(i);
  g_rank = rank;
  g_world = nranks;
  *comm = (void*)(uintptr_t)0xc0;
  logf_("ncclCommInitRank %d %d %s %s", nranks, rank, ok ? "uid-ok" : "uid-bad", hex);
  return ok ? 0 : 4; /* ncclInvalidArgument */
}

int ncclCommDestroy(void* comm) { (void)comm; logf_("ncclCommDestroy"); return 0; }

int ncclAllReduce(const void* send, void* recv, size_t count, int dtype, int op, void* comm, void* stream) {
  (void)comm; (void)stream;
  const int call = g_calls++;
  logf_("ncclAllReduce %zu %d %d", count, dtype, op);
  if (dtype != 4 && dtype != 8) return 4; /* int64 / float64 only */
  const char* dir = getenv("STUB_DIR");
  if (!dir || g_rank < 0) return 3;
  const size_t nb = count * 8;
  char path[4096], tmp[4200];
  snprintf(path, sizeof path, "%s/ar_%d_%d.bin", dir, call, g_rank);
  snprintf(tmp, sizeof tmp, "%s.tmp", path);
  FILE* f = fopen(tmp, "wb");
  if (!f || fwrite(send, 1, nb, f) != nb) return 3;
  fclose(f);
  rename(tmp, path);
  unsigned char* acc = malloc(nb);
  unsigned char* buf = malloc(nb);
  for (int r = 0; r < g_world; ++r) {
    snprintf(path, sizeof path, "%s/ar_%d_%d.bin", dir, call, r);
    int tries = 0;
    for (;;) {
      f = fopen(path, "rb");
      if (f) break;
      if (++tries > 30000) { free(acc); free(buf); return 3; } /* 30 s */
      usleep(1000);
    }
    size_t got = fread(buf, 1, nb, f);
    fclose(f);
    if (got != nb) { free(acc); free(buf); return 3; }
    if (r == 0) { memcpy(acc, buf, nb); continue; }
    for (size_t i = 0; i < count; ++i) {
      if (dtype == 4) {
        int64_t a, b;
        memcpy(&a, acc + 8 * i, 8); memcpy(&b, buf + 8 * i, 8);
        a = op == 0 ? a + b : (a > b ? a : b);
        memcpy(acc + 8 * i, &a, 8);
      } else {
        double a, b;
        memcpy(&a, acc + 8 * i, 8); memcpy(&b, buf + 8 * i, 8);
        a = op == 0 ? a + b : (a > b ? a : b);
        memcpy(acc + 8 * i, &a, 8);
      }
    }
  }
  memcpy(recv, acc, nb);
  free(acc);
  free(buf);
  return 0;
}
