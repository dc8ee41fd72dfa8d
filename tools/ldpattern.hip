// Load-pattern microbenchmark for the LoRA contractions (tools only, not shipped): streams a
// M x K bf16 matrix (M = 14336, K = 2048, 58.7 MB) with the same grid and bytes per wave but
// different per-instruction footprints:
//   P0: 16 rows x 64 B   (lora_down's MFMA-operand layout)
//   P1: 4 rows x 256 B   (lora_wgrad's layout)
//   P2: 2 rows x 512 B   (row-contiguous, as an LDS-staged kernel would load)
// Each thread folds its loads into one value so nothing is dead. Build:
//   hipcc --offload-arch=gfx950 -O3 -o tools/ldpattern tools/ldpattern.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int P>
__global__ __launch_bounds__(512) void ld_kernel(const uint16_t* __restrict__ x, int ldx, float* out) {
  // block: 32 rows, 8 waves each owning 256 columns (lora_down's split)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int m0 = blockIdx.x * 32, k0 = wave * 256;
  uint32_t acc = 0;
  // 16 loads of 16 B per lane cover the wave's 32 x 256 slice
#pragma unroll
  for (int grp = 0; grp < 2; ++grp) {
    u32x4 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int idx = grp * 8 + i;  // 0..15
      int row, col;
      if (P == 0) {  // i -> (row group q = idx & 1, k step st = idx >> 1)
        row = 16 * (idx & 1) + (lane & 15);
        col = 32 * (idx >> 1) + 8 * (lane >> 4);
      } else if (P == 1) {
        row = 4 * (idx & 7) + (lane >> 4);
        col = 128 * (idx >> 3) + 8 * (lane & 15);
      } else {
        row = 2 * idx + (lane >> 5);
        col = 8 * (lane & 31);
      }
      v[i] = *(const u32x4*)(x + (int64_t)(m0 + row) * ldx + k0 + col);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= v[i][0] + v[i][1] + v[i][2] + v[i][3];
  }
  out[blockIdx.x * 512 + threadIdx.x] = (float)acc;
}

// S: grid-stride stream, 1 KB per wave instruction, NL loads in flight per wave
template <int NL>
__global__ __launch_bounds__(256) void stream_kernel(const u32x4* __restrict__ x, int64_t n16, float* out) {
  uint32_t acc = 0;
  const int64_t stride = (int64_t)gridDim.x * 256 * NL;
  for (int64_t i = (int64_t)blockIdx.x * 256 * NL + threadIdx.x; i < n16; i += stride) {
    u32x4 v[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) v[j] = x[min(i + 256 * j, n16 - 1)];
#pragma unroll
    for (int j = 0; j < NL; ++j) acc ^= v[j][0] + v[j][1] + v[j][2] + v[j][3];
  }
  out[blockIdx.x * 256 + threadIdx.x] = (float)acc;
}

// P4: P0 plus lora_down's adapter loads (f32 W[16][K]: per 32-deep k step a lane reads the 8
// weights of its j = lane & 15 at k = kb + 8 * (lane >> 4), served from L2 / L1)
__global__ __launch_bounds__(512) void ldw_kernel(const uint16_t* __restrict__ x, int ldx, const float* __restrict__ W, float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int m0 = blockIdx.x * 32, k0 = wave * 256;
  float facc = 0.f;
  uint32_t acc = 0;
#pragma unroll
  for (int grp = 0; grp < 2; ++grp) {
    u32x4 v[8];
    float4 w[4][2];
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      const int k = k0 + 32 * (grp * 4 + st) + 8 * (lane >> 4);
#pragma unroll
      for (int q = 0; q < 2; ++q) v[st * 2 + q] = *(const u32x4*)(x + (int64_t)(m0 + 16 * q + (lane & 15)) * ldx + k);
      const float* wp = W + (int64_t)(lane & 15) * ldx + k;
      w[st][0] = *(const float4*)wp;
      w[st][1] = *(const float4*)(wp + 4);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= v[i][0] + v[i][1] + v[i][2] + v[i][3];
#pragma unroll
    for (int st = 0; st < 4; ++st) facc += w[st][0].x + w[st][1].w;
  }
  out[blockIdx.x * 512 + threadIdx.x] = (float)acc + facc;
}

// P3: lora_down geometry with all 16 loads of a wave in flight at once
__global__ __launch_bounds__(512) void ld16_kernel(const uint16_t* __restrict__ x, int ldx, float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int m0 = blockIdx.x * 32, k0 = wave * 256;
  uint32_t acc = 0;
  u32x4 v[16];
#pragma unroll
  for (int idx = 0; idx < 16; ++idx)
    v[idx] = *(const u32x4*)(x + (int64_t)(m0 + 16 * (idx & 1) + (lane & 15)) * ldx + k0 + 32 * (idx >> 1) + 8 * (lane >> 4));
#pragma unroll
  for (int i = 0; i < 16; ++i) acc ^= v[i][0] + v[i][1] + v[i][2] + v[i][3];
  out[blockIdx.x * 512 + threadIdx.x] = (float)acc;
}

int main() {
  const int M = 14336, K = 2048;
  uint16_t* x;
  float* out;
  hipMalloc(&x, (size_t)M * K * 2);
  hipMalloc(&out, (size_t)4096 * 512 * 4);  // >= every grid below x block
  hipMemset(x, 1, (size_t)M * K * 2);
  // a 256 MB buffer written between launches so x is not L2/MALL-resident
  char* flush;
  const size_t FL = 256u << 20;
  hipMalloc(&flush, FL);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char* names[3] = {"P0 16 rows x 64 B ", "P1 4 rows x 256 B ", "P2 2 rows x 512 B "};
  for (int hot = 0; hot < 2; ++hot) {
    for (int p = 0; p < 3; ++p) {
      float tot = 0.f;
      const int reps = 50;
      for (int r = 0; r < reps + 5; ++r) {
        if (!hot) hipMemsetAsync(flush, r, FL, 0);
        hipEventRecord(a, 0);
        if (p == 0) hipLaunchKernelGGL(ld_kernel<0>, dim3(M / 32), dim3(512), 0, 0, x, K, out);
        if (p == 1) hipLaunchKernelGGL(ld_kernel<1>, dim3(M / 32), dim3(512), 0, 0, x, K, out);
        if (p == 2) hipLaunchKernelGGL(ld_kernel<2>, dim3(M / 32), dim3(512), 0, 0, x, K, out);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (r >= 5) tot += ms;
      }
      const double us = tot / reps * 1e3;
      printf("%s %s: %.2f us  %.0f GB/s\n", hot ? "hot " : "cold", names[p], us, (double)M * K * 2 / us / 1e3);
    }
  }
  {
    float* W;
    hipMalloc(&W, (size_t)16 * K * 4);
    hipMemset(W, 0, (size_t)16 * K * 4);
    float tot = 0.f;
    const int reps = 50;
    for (int r = 0; r < reps + 5; ++r) {
      hipEventRecord(a, 0);
      hipLaunchKernelGGL(ldw_kernel, dim3(M / 32), dim3(512), 0, 0, x, K, W, out);
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (r >= 5) tot += ms;
    }
    const double us = tot / reps * 1e3;
    printf("hot  P4 P0 + adapter loads : %.2f us  %.0f GB/s (x only)\n", us, (double)M * K * 2 / us / 1e3);
  }
  // hot only: ceilings
  const int64_t n16 = (int64_t)M * K / 8;
  for (int v = 0; v < 7; ++v) {
    float tot = 0.f;
    const int reps = 50;
    const int blocks[7] = {0, 512, 1024, 2048, 1024, 2048, 4096};
    for (int r = 0; r < reps + 5; ++r) {
      hipEventRecord(a, 0);
      if (v == 0) hipLaunchKernelGGL(ld16_kernel, dim3(M / 32), dim3(512), 0, 0, x, K, out);
      else if (v <= 3) hipLaunchKernelGGL(stream_kernel<4>, dim3(blocks[v]), dim3(256), 0, 0, (const u32x4*)x, n16, out);
      else hipLaunchKernelGGL(stream_kernel<8>, dim3(blocks[v]), dim3(256), 0, 0, (const u32x4*)x, n16, out);
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (r >= 5) tot += ms;
    }
    const double us = tot / reps * 1e3;
    if (v == 0) printf("hot  P3 16 loads in flight : %.2f us  %.0f GB/s\n", us, (double)M * K * 2 / us / 1e3);
    else printf("hot  stream NL=%d blocks=%d : %.2f us  %.0f GB/s\n", v <= 3 ? 4 : 8, blocks[v], us, (double)M * K * 2 / us / 1e3);
  }
  return 0;
}
