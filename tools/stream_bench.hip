// Streaming-read microbenchmark for the LoRA kernels' access pattern: how fast can 256 workgroups
// x 8 waves pull a [M, 2048] bf16 matrix (M = 14336, 58.7 MB) through LDS-DMA, by pattern and ring
// depth? Not part of the library.
//   pattern 0 ("tile", lora_dy): wave w of block (cs, rs) owns columns 512 cs + 64 w; a slot is
//             32 rows x 128 B, each DMA instruction 8 rows x 128 B (8 row fragments)
//   pattern 1 ("line"): a slot is 4 rows x 1 KB, each DMA instruction one contiguous 1-KB piece
//             of one row (the block's 8 waves cover 32 rows x 512 columns per stage)
// Operands are cycled over NB buffers (> the 256 MB last-level cache).
// build: hipcc -O3 --offload-arch=gfx950 -o /tmp/stream_bench tools/stream_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

template <int NR, int PAT>
__global__ __launch_bounds__(512) void stream_kernel(const char* __restrict__ y, int ldy_bytes, int M,
                                                     float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) char ring[8][NR][4096];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int cs = blockIdx.x, rs = blockIdx.y;
  const int G = 7;  // slots per wave
  const int mb = rs * G * 32;
  uint32_t off[4];
  const char* base;
  if (PAT == 0) {
    for (int i = 0; i < 4; ++i) off[i] = (uint32_t)((8 * i + (lane >> 3)) * ldy_bytes + (lane & 7) * 16);
    base = y + (size_t)mb * ldy_bytes + (cs * 512 + wave * 64) * 2;
  } else {
    // slot g of wave w: rows mb + 32 g + 4 w + i (i < 4), columns 512 cs .. +512 (1 KB)
    for (int i = 0; i < 4; ++i) off[i] = (uint32_t)(i * ldy_bytes + lane * 16);
    base = y + (size_t)(mb + 4 * wave) * ldy_bytes + cs * 1024;
  }
  const uint32_t lbase = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)&ring[wave][0][0]);
  auto dma = [&](int g) {
    const char* sb = base + (size_t)g * 32 * ldy_bytes;
    const uint32_t l = lbase + (g % NR) * 4096;
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %6\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %5\n\t"
        "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %5\n\t"
        "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %3, %5\n\t"
        "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %4, %5\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(off[0]), "v"(off[1]), "v"(off[2]), "v"(off[3]), "s"(sb), "s"(l)
        : "memory", "scc");
  };
  const int ng = min(G, (M - mb) / 32);
  for (int g = 0; g < NR - 1; ++g)
    if (g < ng) dma(g);
  float acc = 0.f;
  for (int g = 0; g < ng; ++g) {
    const int younger = min(NR - 2, ng - 1 - g);
    if (younger >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (younger == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    acc += *(const float*)&ring[wave][g % NR][lane * 64];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (g + NR - 1 < ng) dma(g + NR - 1);
  }
  if (acc == 12345.f) out[threadIdx.x] = acc;  // keeps the reads
}

int main() {
  const int M = 14336, N = 2048, NB = 6;
  const size_t bytes = (size_t)M * N * 2;
  std::vector<char*> bufs(NB);
  for (auto& b : bufs) {
    hipMalloc(&b, bytes);
    hipMemset(b, 1, bytes);
  }
  float* out;
  hipMalloc(&out, 4096);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const dim3 grid(4, M / (7 * 32));
  auto run = [&](auto kern, const char* name) {
    for (int i = 0; i < NB; ++i) kern<<<grid, 512>>>(bufs[i], N * 2, M, out);
    hipDeviceSynchronize();
    const int it = 60;
    hipEventRecord(e0);
    for (int i = 0; i < it; ++i) kern<<<grid, 512>>>(bufs[i % NB], N * 2, M, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / it;
    printf("%-12s %7.2f us  %6.2f TB/s\n", name, us, bytes / us / 1e6);
  };
  run(stream_kernel<3, 0>, "tile nr3");
  run(stream_kernel<4, 0>, "tile nr4");
  run(stream_kernel<5, 0>, "tile nr5");
  run(stream_kernel<3, 1>, "line nr3");
  run(stream_kernel<4, 1>, "line nr4");
  run(stream_kernel<5, 1>, "line nr5");
  return 0;
}
