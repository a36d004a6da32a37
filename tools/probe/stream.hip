// Streaming-bandwidth calibration for the W-MSA forward byte mix (3 bytes read : 1 written).
//   hipcc --offload-arch=gfx950 -O3 stream.hip -o stream && ./stream
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(err_)); return 1; } } while (0)

// one-shot: each thread moves 3 float4 in, 1 float4 out (rows of 3 float4 -> 1)
typedef float f4v __attribute__((ext_vector_type(4)));
template <bool NT>
__global__ __launch_bounds__(256) void oneshot(const f4v* __restrict__ in, f4v* __restrict__ out, size_t n_out) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n_out) return;
  f4v a, b, c;
  if (NT) {
    a = __builtin_nontemporal_load(in + i);
    b = __builtin_nontemporal_load(in + i + n_out);
    c = __builtin_nontemporal_load(in + i + 2 * n_out);
  } else {
    a = in[i]; b = in[i + n_out]; c = in[i + 2 * n_out];
  }
  f4v r = a + b + c;
  if (NT) __builtin_nontemporal_store(r, out + i); else out[i] = r;
}

// persistent grid-stride with UNROLL independent iterations in flight per thread
template <int UNROLL>
__global__ __launch_bounds__(256) void persist(const float4* __restrict__ in, float4* __restrict__ out, size_t n_out) {
  const size_t stride = (size_t)gridDim.x * 256;
  for (size_t base = (size_t)blockIdx.x * 256 + threadIdx.x; base < n_out; base += stride * UNROLL) {
    float4 v[UNROLL][3];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const size_t i = base + u * stride;
      if (i < n_out) { v[u][0] = in[i]; v[u][1] = in[i + n_out]; v[u][2] = in[i + 2 * n_out]; }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const size_t i = base + u * stride;
      if (i < n_out)
        out[i] = make_float4(v[u][0].x + v[u][1].x + v[u][2].x, v[u][0].y + v[u][1].y + v[u][2].y,
                             v[u][0].z + v[u][1].z + v[u][2].z, v[u][0].w + v[u][1].w + v[u][2].w);
    }
  }
}

// W-MSA-shaped gather: a wave owns 16 rows of a [T, 3C] bf16 tensor and reads a 64-B slice of
// q, k, v (16 B per lane) for one head, writes 64 B per row of [T, C]; rows in a shuffled-window
// order within 7-row bands like the real kernel (row = window-local t mapping).
template <bool NT>
__global__ __launch_bounds__(256) void gather64(const uint4* __restrict__ qkv, uint4* __restrict__ out, int T, int C, int nH) {
  const int wave = (blockIdx.x * 256 + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  const int tiles = T / 16;
  const int nwaves = gridDim.x * 4;
  const int li = lane & 15, g = lane >> 4;
  const int C3u = 3 * C / 8, Cu = C / 8;  // uint4 per row
  for (int w = wave; w < tiles * nH; w += nwaves * 4) {
    uint4 v[4][3];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ww = w + u * nwaves;
      if (ww < tiles * nH) {
        const int h = ww % nH, tile = ww / nH;
        const size_t row = (size_t)tile * 16 + li;
        const uint4* p = qkv + row * C3u + h * 4 + g;
        if (NT) {
          typedef unsigned int u4 __attribute__((ext_vector_type(4)));
          const u4* q = reinterpret_cast<const u4*>(p);
          v[u][0] = __builtin_bit_cast(uint4, __builtin_nontemporal_load(q));
          v[u][1] = __builtin_bit_cast(uint4, __builtin_nontemporal_load(q + Cu));
          v[u][2] = __builtin_bit_cast(uint4, __builtin_nontemporal_load(q + 2 * Cu));
        } else {
          v[u][0] = p[0]; v[u][1] = p[Cu]; v[u][2] = p[2 * Cu];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ww = w + u * nwaves;
      if (ww < tiles * nH) {
        const int h = ww % nH, tile = ww / nH;
        const size_t row = (size_t)tile * 16 + li;
        uint4 r = v[u][0];
        r.x ^= v[u][1].x ^ v[u][2].x; r.y ^= v[u][1].y ^ v[u][2].y;
        r.z ^= v[u][1].z ^ v[u][2].z; r.w ^= v[u][1].w ^ v[u][2].w;
        if (NT) {
          typedef unsigned int u4 __attribute__((ext_vector_type(4)));
          __builtin_nontemporal_store(__builtin_bit_cast(u4, r), reinterpret_cast<u4*>(out + row * Cu + h * 4 + g));
        } else {
          out[row * Cu + h * 4 + g] = r;
        }
      }
    }
  }
}

int main() {
  const int T = 256 * 56 * 56, C = 96;
  const size_t in_bytes = (size_t)T * 3 * C * 2, out_bytes = (size_t)T * C * 2;  // stage-0 sizes
  const size_t n_out = out_bytes / 16;
  void *in, *out;
  CK(hipMalloc(&in, in_bytes));
  CK(hipMalloc(&out, out_bytes));
  CK(hipMemset(in, 0, in_bytes));
  hipEvent_t s = nullptr, e = nullptr;
  CK(hipEventCreate(&s)); CK(hipEventCreate(&e));
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    (void)hipEventRecord(s);
    const int it = 20;
    for (int i = 0; i < it; ++i) launch();
    (void)hipEventRecord(e);
    (void)hipEventSynchronize(e);
    float ms; (void)hipEventElapsedTime(&ms, s, e);
    ms /= it;
    printf("%-28s %8.1f us  %7.0f GB/s\n", name, ms * 1e3, (in_bytes + out_bytes) / ms / 1e6);
  };
  const float4* i4 = (const float4*)in; float4* o4 = (float4*)out;
  const int blocks = (int)((n_out + 255) / 256);
  run("oneshot", [&] { hipLaunchKernelGGL(oneshot<false>, dim3(blocks), dim3(256), 0, 0, (const f4v*)in, (f4v*)out, n_out); });
  run("oneshot-nt", [&] { hipLaunchKernelGGL(oneshot<true>, dim3(blocks), dim3(256), 0, 0, (const f4v*)in, (f4v*)out, n_out); });
  for (int g : {1024, 2048, 4096})
    for (int u : {1, 2, 4}) {
      char nm[64]; snprintf(nm, 64, "persist g=%d u=%d", g, u);
      run(nm, [&] {
        if (u == 1) hipLaunchKernelGGL(persist<1>, dim3(g), dim3(256), 0, 0, i4, o4, n_out);
        if (u == 2) hipLaunchKernelGGL(persist<2>, dim3(g), dim3(256), 0, 0, i4, o4, n_out);
        if (u == 4) hipLaunchKernelGGL(persist<4>, dim3(g), dim3(256), 0, 0, i4, o4, n_out);
      });
    }
  for (int g : {1024, 4096, 16384}) {
    char nm[64]; snprintf(nm, 64, "gather64 g=%d", g);
    run(nm, [&] { hipLaunchKernelGGL(gather64<false>, dim3(g), dim3(256), 0, 0, (const uint4*)in, (uint4*)out, T, C, 3); });
    snprintf(nm, 64, "gather64-nt g=%d", g);
    run(nm, [&] { hipLaunchKernelGGL(gather64<true>, dim3(g), dim3(256), 0, 0, (const uint4*)in, (uint4*)out, T, C, 3); });
  }
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  return 0;
}
