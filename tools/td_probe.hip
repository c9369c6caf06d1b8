// td_probe.hip — vector-memory gather throughput on one MI355X (round-5 measurement for the traversal's record
// fetches): every wave of a persistent grid (one 1024-thread workgroup per CU, like k_traverse) issues dependent
// chains of 16-byte (or 8-byte) gathers from a table, with a chosen number of active lanes and a chosen number
// of distinct cache lines per instruction.  Prints ns per wave-instruction and per active lane.
// build: hipcc --offload-arch=gfx950 -O3 -o td_probe tools/td_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                             \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
      std::exit(1);                                                          \
    }                                                                        \
  } while (0)

// table: n16 16-byte records; next index = f(record contents) so the chain is dependent (as a walk is)
template <int BYTES>
__global__ __launch_bounds__(1024) void k_gather(const uint4* __restrict__ table, uint32_t mask, int steps, int active,
                                                 int lines, uint32_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  uint32_t acc = 0;
  if (lane < active) {
    // lanes in groups of 64 / lines share a cache line (8 records of 16 bytes), each lane its own record in it
    const int grp = lines >= 64 ? lane : lane / (64 / lines);
    const uint32_t sub = lines >= 64 ? 0u : (uint32_t)(lane & 7);
    uint32_t idx[4];
#pragma unroll
    for (int c = 0; c < 4; c++) idx[c] = (blockIdx.x * 64u + (threadIdx.x >> 6) * 131u + grp * 977u + c * 7919u) * 2654435761u;
    for (int s = 0; s < steps; s++) {
#pragma unroll
      for (int c = 0; c < 4; c++) {  // four independent chains per lane
        const uint32_t i = lines >= 64 ? (idx[c] & mask) : (((idx[c] & mask) & ~7u) | sub);
        if constexpr (BYTES == 16) {
          const uint4 r = table[i];
          acc += r.x ^ r.w;
          idx[c] = idx[c] * 1664525u + 1013904223u + (r.y & 1u);
        } else {
          const uint2 r = reinterpret_cast<const uint2*>(table)[2 * i];
          acc += r.x;
          idx[c] = idx[c] * 1664525u + 1013904223u + (r.y & 1u);
        }
      }
    }
  }
  if (acc == 0xFFFFFFFFu) out[threadIdx.x] = acc;
}

int main(int argc, char** argv) {
  const int steps = 2000;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int n_cu = prop.multiProcessorCount;
  uint32_t* out;
  CHECK(hipMalloc(&out, 4096 * 4));
  for (int tbl_kb : {16, 256, 2048, 16384}) {
    const size_t n16 = (size_t)tbl_kb * 1024 / 16;
    std::vector<uint4> h(n16);
    for (size_t i = 0; i < n16; i++) h[i] = make_uint4((uint32_t)i * 7u, (uint32_t)(i * 2654435761u), 3u, 5u);
    uint4* t;
    CHECK(hipMalloc(&t, n16 * 16));
    CHECK(hipMemcpy(t, h.data(), n16 * 16, hipMemcpyHostToDevice));
    const uint32_t mask = (uint32_t)n16 - 1;
    for (int bytes : {16, 8})
      for (int active : {64, 32, 8})
        for (int lines : {64, 8, 1}) {
          if (lines > active) continue;
          hipEvent_t a, b;
          CHECK(hipEventCreate(&a));
          CHECK(hipEventCreate(&b));
          for (int rep = 0; rep < 2; rep++) {
            CHECK(hipEventRecord(a));
            if (bytes == 16) k_gather<16><<<n_cu, 1024>>>(t, mask, steps, active, lines, out);
            else k_gather<8><<<n_cu, 1024>>>(t, mask, steps, active, lines, out);
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
          }
          float ms = 0;
          CHECK(hipEventElapsedTime(&ms, a, b));
          const double instr_per_cu = 16.0 * 4 * steps;  // 16 waves per CU, 4 loads per step
          const double ns_per_instr = ms * 1e6 / instr_per_cu;
          std::printf("{\"table_kb\": %d, \"bytes\": %d, \"active\": %d, \"lines\": %d, \"ms\": %.3f, "
                      "\"ns_per_wave_instr_per_cu\": %.3f, \"ns_per_lane\": %.4f}\n",
                      tbl_kb, bytes, active, lines, ms, ns_per_instr, ns_per_instr / active);
          CHECK(hipEventDestroy(a));
          CHECK(hipEventDestroy(b));
        }
    CHECK(hipFree(t));
  }
  return 0;
}
