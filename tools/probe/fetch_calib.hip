// FETCH_SIZE / WRITE_SIZE calibration on gfx950 (MI355X_MICROARCH.md: "other access widths
// are uncalibrated: calibrate on a known byte count in your own access pattern").  Each
// kernel touches every byte of a 1 GiB buffer exactly once (4x the 256 MB Infinity Cache),
// in one access shape; rocprofv3 --pmc FETCH_SIZE (or WRITE_SIZE) per dispatch / the known
// byte count is the correction factor for that shape:
//   rd16 / rd8 / rd4     coalesced streaming loads of 16 / 8 / 4 B per lane
//   seg64                the W-MSA fragment shape: one 16-B load per lane, lanes = 16 rows x
//                        4 units of one 64-B head segment, rows 576 B apart (stage-0 qkv),
//                        every segment of every row read once across the grid
//   dma16                global_load_lds_dwordx4 (LDS-DMA) streaming, 1 KiB per wave-instruction
//   wr16 / wr8 / wseg64  the same shapes as stores
//   timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d OUT -o run --output-format csv -- ./fetch_calib
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(err_)); return 1; } } while (0)

constexpr size_t BYTES = 1ull << 30;
constexpr int ROWB = 576;  // stage-0 qkv row bytes (3C bf16, C = 96)

template <typename T>
__global__ __launch_bounds__(256) void rd(const T* __restrict__ p, unsigned* __restrict__ out, size_t n) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const T v = p[i];
    acc ^= reinterpret_cast<const unsigned*>(&v)[0];
  }
  if (acc == 0x12345678u) out[0] = acc;  // never true: keeps the loads
}

template <typename T>
__global__ __launch_bounds__(256) void wr(T* __restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    T v;
    reinterpret_cast<unsigned*>(&v)[0] = (unsigned)i;
    for (int k = 1; k < (int)(sizeof(T) / 4); ++k) reinterpret_cast<unsigned*>(&v)[k] = 0;
    p[i] = v;
  }
}

// wave w handles (row block rb, segment s): 16 rows x 64 B
__global__ __launch_bounds__(256) void seg64(const char* __restrict__ p, unsigned* __restrict__ out, int nrb) {
  const int lane = threadIdx.x & 63, li = lane & 15, gq = lane >> 4;
  const int nseg = ROWB / 64;
  unsigned acc = 0;
  for (int u = blockIdx.x * 4 + (threadIdx.x >> 6); u < nrb * nseg; u += gridDim.x * 4) {
    const int rb = u / nseg, s = u % nseg;
    const uint4 v = *reinterpret_cast<const uint4*>(p + (size_t)(16 * rb + li) * ROWB + 64 * s + 16 * gq);
    acc ^= v.x;
  }
  if (acc == 0x12345678u) out[0] = acc;
}
__global__ __launch_bounds__(256) void wseg64(char* __restrict__ p, int nrb) {
  const int lane = threadIdx.x & 63, li = lane & 15, gq = lane >> 4;
  const int nseg = ROWB / 64;
  for (int u = blockIdx.x * 4 + (threadIdx.x >> 6); u < nrb * nseg; u += gridDim.x * 4) {
    const int rb = u / nseg, s = u % nseg;
    *reinterpret_cast<uint4*>(p + (size_t)(16 * rb + li) * ROWB + 64 * s + 16 * gq) = make_uint4(u, 0, 0, 0);
  }
}

typedef __attribute__((address_space(3))) void* lds_vptr;
typedef __attribute__((address_space(1))) void* gbl_vptr;
__global__ __launch_bounds__(256) void dma16(const char* __restrict__ p, unsigned* __restrict__ out, size_t n) {
  __shared__ __attribute__((aligned(16))) char buf[4 * 1024];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (size_t c = (size_t)blockIdx.x * 4 + wave; c < n / 1024; c += (size_t)gridDim.x * 4)
    __builtin_amdgcn_global_load_lds((gbl_vptr)(p + c * 1024 + 16 * lane), (lds_vptr)(buf + wave * 1024), 16, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (buf[threadIdx.x] == 123 && threadIdx.x == 0x7fff) out[0] = 1;
}

int main() {
  char* buf;
  unsigned* out;
  CK(hipMalloc(&buf, BYTES));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(buf, 1, BYTES));
  // a 1 GiB sweep of another buffer between kernels flushes the caches
  char* flush;
  CK(hipMalloc(&flush, BYTES));
  auto fl = [&] { hipLaunchKernelGGL(wr<uint4>, dim3(8192), dim3(256), 0, 0, (uint4*)flush, BYTES / 16); };
  const int grid = 8192;
  const int nrb = (int)(BYTES / ROWB / 16);
  fl(); hipLaunchKernelGGL(rd<uint4>, dim3(grid), dim3(256), 0, 0, (const uint4*)buf, out, BYTES / 16);
  fl(); hipLaunchKernelGGL(rd<uint2>, dim3(grid), dim3(256), 0, 0, (const uint2*)buf, out, BYTES / 8);
  fl(); hipLaunchKernelGGL(rd<unsigned>, dim3(grid), dim3(256), 0, 0, (const unsigned*)buf, out, BYTES / 4);
  fl(); hipLaunchKernelGGL(seg64, dim3(grid), dim3(256), 0, 0, (const char*)buf, out, nrb);
  fl(); hipLaunchKernelGGL(dma16, dim3(grid), dim3(256), 0, 0, (const char*)buf, out, BYTES);
  fl(); hipLaunchKernelGGL(wr<uint4>, dim3(grid), dim3(256), 0, 0, (uint4*)buf, BYTES / 16);
  fl(); hipLaunchKernelGGL(wr<uint2>, dim3(grid), dim3(256), 0, 0, (uint2*)buf, BYTES / 8);
  fl(); hipLaunchKernelGGL(wseg64, dim3(grid), dim3(256), 0, 0, buf, nrb);
  CK(hipDeviceSynchronize());
  printf("known bytes: streaming kernels %zu, seg64 kernels %zu\n", BYTES, (size_t)nrb * 16 * ROWB);
  return 0;
}
