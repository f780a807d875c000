// Probe (measurement tool, not product code): what a wave-uniform 16-byte LDS
// store costs when every lane stores the same bytes (the engine's serial
// EMIT into the option buffer, and every scalar field write of the game row)
// against the same store from lane 0 only.  One 64-lane workgroup per wave,
// W waves per SIMD; each wave stores N options into its own 64-entry buffer
// and reads one back so the stores are not dead.
//   hipcc --offload-arch=gfx950 -O3 tools/lds_store_probe.hip -o build/lds_store_probe
//   build/lds_store_probe            -> one line per (mode, waves per SIMD)
#include <hip/hip_runtime.h>

#include <cstdio>

struct Opt {
  uint32_t w[4];
};

// MODE 0: 16 B, every lane the same address (a serial EMIT); 1: the same from
// lane 0 only; 2: 16 B, every lane its own slot; 3: 4 B every lane the same
// address (a field write); 4: 1 B the same; 5: 4 B every lane its own dword.
template <int MODE>
__global__ __launch_bounds__(64) void k_probe(int n, uint32_t seed, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint4 buf[128];
  const int lane = threadIdx.x;
  uint32_t x = seed ^ blockIdx.x;
  uint32_t* b32 = reinterpret_cast<uint32_t*>(buf);
  uint8_t* b8 = reinterpret_cast<uint8_t*>(buf);
#pragma nounroll
  for (int i = 0; i < n; i++) {
    x = x * 1664525u + 1013904223u;                       // wave-uniform value
    const uint4 v = make_uint4(x, x ^ 1u, x ^ 2u, x ^ 3u);
    if (MODE == 0) buf[i & 127] = v;
    else if (MODE == 1) { if (lane == 0) buf[i & 127] = v; }
    else if (MODE == 2) buf[(i + lane) & 127] = v;
    else if (MODE == 3) b32[i & 511] = x;
    else if (MODE == 4) b8[i & 2047] = (uint8_t)x;
    else b32[(i + lane) & 511] = x;
  }
  __syncthreads();
  uint4 r = buf[(x >> 3) & 127];
  if (lane == 0) out[blockIdx.x] = r.x + r.y + r.z + r.w;
}

int main() {
  const int n = 4096, cus = 256;
  uint32_t* out;
  hipMalloc(&out, sizeof(uint32_t) * cus * 32);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int w = 1; w <= 8; w *= 2) {
    const int blocks = cus * 4 * w;
    for (int mode = 0; mode < 6; mode++) {
      float best = 1e9f;
      for (int rep = 0; rep < 4; rep++) {
        hipEventRecord(a);
        if (mode == 0) hipLaunchKernelGGL(k_probe<0>, dim3(blocks), dim3(64), 0, 0, n, 7u, out);
        if (mode == 1) hipLaunchKernelGGL(k_probe<1>, dim3(blocks), dim3(64), 0, 0, n, 7u, out);
        if (mode == 2) hipLaunchKernelGGL(k_probe<2>, dim3(blocks), dim3(64), 0, 0, n, 7u, out);
        if (mode == 3) hipLaunchKernelGGL(k_probe<3>, dim3(blocks), dim3(64), 0, 0, n, 7u, out);
        if (mode == 4) hipLaunchKernelGGL(k_probe<4>, dim3(blocks), dim3(64), 0, 0, n, 7u, out);
        if (mode == 5) hipLaunchKernelGGL(k_probe<5>, dim3(blocks), dim3(64), 0, 0, n, 7u, out);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (rep && ms < best) best = ms;
      }
      // cycles per store per wave at 2.4 GHz: the kernel time over the stores one wave issues
      printf("{\"mode\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"cycles_per_store_per_wave\": %.1f}\n",
             mode == 0 ? "b128_same_addr" : mode == 1 ? "b128_lane0_only" : mode == 2 ? "b128_own_addr"
             : mode == 3 ? "b32_same_addr" : mode == 4 ? "b8_same_addr" : "b32_own_addr", w, best,
             best * 1e-3 * 2.4e9 / n);
    }
  }
  hipFree(out);
  return 0;
}
