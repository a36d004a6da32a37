// Store-pattern probe: HBM write rate of the skinny GEMM's output shape (16 rows x 64 B per
// wave instruction, 16 B per lane) against row-contiguous 1 KB per instruction, and the same
// for loads.  ./store_pattern  -> one line per pattern (GB/s).
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int ROWLEN = 768;  // bytes per row (384 bf16 columns), as the stage-0 fc1 output

// pattern A: lane (li, g) writes row 16t + li, bytes 64j + 16g .. +15, j = 0 .. ROWLEN/64-1
__global__ void st_frag(uint4* __restrict__ out, int tiles) {
  const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
  const int wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int nw = gridDim.x * (blockDim.x >> 6);
  for (int t = wave; t < tiles; t += nw) {
    char* row = reinterpret_cast<char*>(out) + (size_t)(16 * t + li) * ROWLEN;
#pragma unroll
    for (int j = 0; j < ROWLEN / 64; ++j)
      *reinterpret_cast<uint4*>(row + 64 * j + 16 * g) = make_uint4(t, j, lane, 1);
  }
}
// pattern B: the same 16-row tile written as whole rows, 1 KB contiguous per instruction
__global__ void st_rows(uint4* __restrict__ out, int tiles) {
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int nw = gridDim.x * (blockDim.x >> 6);
  for (int t = wave; t < tiles; t += nw) {
    char* base = reinterpret_cast<char*>(out) + (size_t)16 * t * ROWLEN;
#pragma unroll
    for (int j = 0; j < 16 * ROWLEN / 1024; ++j)
      *reinterpret_cast<uint4*>(base + 1024 * j + 16 * lane) = make_uint4(t, j, lane, 1);
  }
}
__global__ void ld_frag(const uint4* __restrict__ in, int tiles, uint4* sink) {
  const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
  const int wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int nw = gridDim.x * (blockDim.x >> 6);
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (int t = wave; t < tiles; t += nw) {
    const char* row = reinterpret_cast<const char*>(in) + (size_t)(16 * t + li) * ROWLEN;
#pragma unroll
    for (int j = 0; j < ROWLEN / 64; ++j) {
      const uint4 v = *reinterpret_cast<const uint4*>(row + 64 * j + 16 * g);
      acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
  }
  if (acc.x == 0x12345678u) sink[0] = acc;
}
__global__ void ld_rows(const uint4* __restrict__ in, int tiles, uint4* sink) {
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int nw = gridDim.x * (blockDim.x >> 6);
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (int t = wave; t < tiles; t += nw) {
    const char* base = reinterpret_cast<const char*>(in) + (size_t)16 * t * ROWLEN;
#pragma unroll
    for (int j = 0; j < 16 * ROWLEN / 1024; ++j) {
      const uint4 v = *reinterpret_cast<const uint4*>(base + 1024 * j + 16 * lane);
      acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
  }
  if (acc.x == 0x12345678u) sink[0] = acc;
}

int main() {
  const int tiles = 802816 / 16;
  const size_t bytes = (size_t)tiles * 16 * ROWLEN;
  uint4 *buf, *sink;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int grids[] = {256, 512, 1024, 2048};
  for (int p = 0; p < 4; ++p)
    for (int gi = 0; gi < 4; ++gi) {
      const int grid = grids[gi];
      auto run = [&]() {
        if (p == 0) hipLaunchKernelGGL(st_frag, dim3(grid), dim3(512), 0, 0, buf, tiles);
        if (p == 1) hipLaunchKernelGGL(st_rows, dim3(grid), dim3(512), 0, 0, buf, tiles);
        if (p == 2) hipLaunchKernelGGL(ld_frag, dim3(grid), dim3(512), 0, 0, buf, tiles, sink);
        if (p == 3) hipLaunchKernelGGL(ld_rows, dim3(grid), dim3(512), 0, 0, buf, tiles, sink);
      };
      for (int i = 0; i < 3; ++i) run();
      hipEventRecord(e0, 0);
      for (int i = 0; i < 10; ++i) run();
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const char* names[] = {"store 16 rows x 64 B", "store 1 KB rows", "load 16 rows x 64 B",
                             "load 1 KB rows"};
      printf("%-22s grid %5d: %7.1f us  %6.0f GB/s\n", names[p], grid, ms * 100, bytes / (ms / 10 * 1e-3) / 1e9);
    }
  return 0;
}
