// Standalone check of the TCP fast-retransmit walk's loop shape (tgsim_tcp.hip, k_tcp_conn_release,
// VERDICT r5 item 7): per lane a walk along a linked list that stops at the list head or at the third
// ACKed segment, then a test of the count after the loop. Lanes of one wave walk different lengths.
// WALK_ASM=1 passes the count through an empty asm (the product's form), 0 leaves it to the compiler.
// Prints the lanes whose post-loop decision differs from the host's.
//   hipcc --offload-arch=gfx950 -O3 -DWALK_ASM=0 tools/loopexit_repro.hip -o /tmp/walk0
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#ifndef WALK_ASM
#define WALK_ASM 0
#endif

__global__ void walk(const uint32_t* next, const uint8_t* done, const uint32_t* una, const uint32_t* head,
                     const uint8_t* broken, const uint32_t* fr, const uint32_t* state, uint32_t* out, uint32_t n) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  uint32_t res = 0xFFFFFFFFu;
  const uint32_t h0 = head[k];
  uint32_t u = una[k];
  while (u != h0 && done[u]) u = next[u];
  if (u != h0 && !broken[k] && fr[k] != u) {
    const uint32_t ws = state[k];
    uint32_t dup = 0;
    for (uint32_t x = next[u]; x != h0 && dup < 3u; x = next[x]) dup += done[x] == 1;
#if WALK_ASM
    __asm__ volatile("" : "+v"(dup));
#endif
    if (dup >= 3u && ws != 5u && ws != 6u) res = u;
    else res = 0xFFFFFFFEu;
  }
  out[k] = res;
}

int main() {
  const uint32_t n = 1 << 16, per = 24;          // n lists of `per` segments each
  std::vector<uint32_t> next(n * per + 1), una(n), head(n), fr(n), state(n), want(n), got(n);
  std::vector<uint8_t> done(n * per + 1), broken(n);
  srand(7);
  const uint32_t end = n * per;                  // a shared terminator (the list head past the tail)
  for (uint32_t k = 0; k < n; ++k) {
    const uint32_t len = 1 + rand() % per;       // each lane walks its own length
    for (uint32_t i = 0; i < len; ++i) {
      const uint32_t s = k * per + i;
      next[s] = i + 1 < len ? s + 1 : end;
      done[s] = (rand() % 3) == 0 ? 1 : ((rand() % 7) == 0 ? 2 : 0);
    }
    una[k] = k * per;
    head[k] = end;
    broken[k] = (rand() % 17) == 0;
    fr[k] = (rand() % 13) == 0 ? k * per : 0xFFFFFFFFu;
    state[k] = rand() % 8;
  }
  done[end] = 0;
  next[end] = end;
  for (uint32_t k = 0; k < n; ++k) {  // the host's answer
    uint32_t res = 0xFFFFFFFFu, u = una[k];
    const uint32_t h0 = head[k];
    while (u != h0 && done[u]) u = next[u];
    if (u != h0 && !broken[k] && fr[k] != u) {
      uint32_t dup = 0;
      for (uint32_t x = next[u]; x != h0 && dup < 3u; x = next[x]) dup += done[x] == 1;
      res = (dup >= 3u && state[k] != 5u && state[k] != 6u) ? u : 0xFFFFFFFEu;
    }
    want[k] = res;
  }
  uint32_t *dn, *du, *dh, *dfr, *ds, *dout;
  uint8_t *dd, *db;
  hipMalloc(&dn, next.size() * 4); hipMalloc(&dd, done.size()); hipMalloc(&du, n * 4); hipMalloc(&dh, n * 4);
  hipMalloc(&db, n); hipMalloc(&dfr, n * 4); hipMalloc(&ds, n * 4); hipMalloc(&dout, n * 4);
  hipMemcpy(dn, next.data(), next.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dd, done.data(), done.size(), hipMemcpyHostToDevice);
  hipMemcpy(du, una.data(), n * 4, hipMemcpyHostToDevice);
  hipMemcpy(dh, head.data(), n * 4, hipMemcpyHostToDevice);
  hipMemcpy(db, broken.data(), n, hipMemcpyHostToDevice);
  hipMemcpy(dfr, fr.data(), n * 4, hipMemcpyHostToDevice);
  hipMemcpy(ds, state.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(walk, dim3(n / 256), dim3(256), 0, 0, dn, dd, du, dh, db, dfr, ds, dout, n);
  if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 2; }
  hipMemcpy(got.data(), dout, n * 4, hipMemcpyDeviceToHost);
  uint32_t bad = 0, fast = 0;
  for (uint32_t k = 0; k < n; ++k) {
    bad += got[k] != want[k];
    fast += want[k] < 0xFFFFFFFEu;
  }
  printf("WALK_ASM=%d lanes %u fast-retransmits expected %u mismatches %u\n", WALK_ASM, n, fast, bad);
  return bad ? 1 : 0;
}
