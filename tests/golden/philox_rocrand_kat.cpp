// Generates Philox4x32-10 known-answer vectors from rocRAND's host-callable engine
// (/opt/rocm/include/rocrand/rocrand_philox4x32_10.h, philox4x32_10_engine::ten_rounds), an
// implementation independent of both the oracle and the HIP kernels. Built and run by
// tests/golden/make_golden.py; output committed as tests/golden/philox_rocrand.json.
#include <cstdio>
#include <cstdint>
#include <rocrand/rocrand_philox4x32_10.h>

struct Engine : rocrand_device::philox4x32_10_engine {
  Engine() : rocrand_device::philox4x32_10_engine(0, 0, 0) {}
  using rocrand_device::philox4x32_10_engine::ten_rounds;  // protected in the engine
};

int main() {
  Engine e;
  uint64_t s = 0x9E3779B97F4A7C15ull;
  auto next = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (uint32_t)s; };
  std::printf("[\n");
  for (int i = 0; i < 64; ++i) {
    uint4 c;
    uint2 k;
    if (i == 0) { c = uint4{0, 0, 0, 0}; k = uint2{0, 0}; }
    else if (i == 1) { c = uint4{~0u, ~0u, ~0u, ~0u}; k = uint2{~0u, ~0u}; }
    else { c = uint4{next(), next(), next(), next()}; k = uint2{next(), next()}; }
    uint4 o = e.ten_rounds(c, k);
    std::printf("  {\"ctr\": [%u, %u, %u, %u], \"key\": [%u, %u], \"out\": [%u, %u, %u, %u]}%s\n",
                c.x, c.y, c.z, c.w, k.x, k.y, o.x, o.y, o.z, o.w, i == 63 ? "" : ",");
  }
  std::printf("]\n");
  return 0;
}
