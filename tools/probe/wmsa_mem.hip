// Memory-shape probe for the W-MSA forward at the SwinV2-T stage-0 shape (T = 256*56*56,
// C = 96, 3 heads, window 7, shift 3): the forward's bytes (read qkv [T,3C] bf16, write
// out [T,C] bf16) moved with no attention math, in two access shapes:
//   frag  - one wave per (window, head): 16 rows x 64 B per load instruction (the round-1
//           kernel's shape), persistent 4 workgroups/CU
//   slab  - one workgroup per window chunk, all heads: the window's 7 row runs (4 KB each)
//           staged whole into an LDS ring by global_load_lds (full lines), each wave reads its
//           head's fragments from LDS (ds_read_b128), the output goes back through the q
//           slots of the slab and leaves as contiguous row runs.
// A fake VALU loop of D iterations per (window, head) emulates the attention math.
//   hipcc --offload-arch=gfx950 -O3 wmsa_mem.hip -o wmsa_mem && ./wmsa_mem
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(err_)); return 1; } } while (0)

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

struct Geom { int B, H, W, C, nH, win, shift, nWh, nWw, nwin; };

__device__ __forceinline__ int token_row(const Geom& g, int w, int t) {
  const int per = g.nWh * g.nWw;
  const int b = w / per, rem = w % per, wh = rem / g.nWw, ww = rem % g.nWw;
  int y = wh * g.win + t / g.win + g.shift, x = ww * g.win + t % g.win + g.shift;
  if (y >= g.H) y -= g.H;
  if (x >= g.W) x -= g.W;
  return (b * g.H + y) * g.W + x;
}

__device__ __forceinline__ float fake_math(uint4 v, int D) {
  float a = __uint_as_float(v.x & 0x3f800000u), b = __uint_as_float(v.y | 0x3f800000u);
  for (int i = 0; i < D; ++i) { a = __builtin_fmaf(a, b, 1.0f); b = __builtin_fmaf(b, a, -1.0f); }
  return a + b;
}

// ---- frag: round-1 shape
__global__ __launch_bounds__(256, 4) void frag(const uint4* __restrict__ qkv, uint4* __restrict__ out, Geom g, int chunks, int D) {
  const int h = blockIdx.x % g.nH, chunk = blockIdx.x / g.nH;
  const int w0 = (int)((long long)chunk * g.nwin / chunks), w1 = (int)((long long)(chunk + 1) * g.nwin / chunks);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, gq = lane >> 4;
  const int C3u = 3 * g.C / 8, Cu = g.C / 8;
  for (int w = w0 + wave; w < w1; w += 4) {
    uint4 q[4], k[4], v[4];
    int row[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = 16 * i + li;
      row[i] = token_row(g, w, t < 49 ? t : 0);
      if (t < 49) {
        const uint4* p = qkv + (size_t)row[i] * C3u + h * 4 + gq;
        q[i] = p[0]; k[i] = p[Cu]; v[i] = p[2 * Cu];
      } else q[i] = k[i] = v[i] = make_uint4(0, 0, 0, 0);
    }
    float f = fake_math(q[0], D);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (16 * i + li < 49) {
        uint4 r = q[i];
        r.x ^= k[i].x ^ v[i].x ^ __float_as_uint(f); r.y ^= k[i].y ^ v[i].y; r.z ^= k[i].z ^ v[i].z; r.w ^= k[i].w ^ v[i].w;
        out[(size_t)row[i] * Cu + h * 4 + gq] = r;
      }
  }
}

// ---- slab: full-row glds staging, HG = nH heads per workgroup, one wave per head
template <int NBUF>
__global__ __launch_bounds__(192, 1) void slab(const char* __restrict__ qkv, char* __restrict__ out, Geom g, int chunks, int D) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int chunk = blockIdx.x;
  const int w0 = (int)((long long)chunk * g.nwin / chunks), w1 = (int)((long long)(chunk + 1) * g.nwin / chunks);
  const int N = g.win * g.win;
  const int rowslots = 3 * g.C / 8;             // 16-B slots per token row (36 at C=96)
  const int slabslots = N * rowslots;           // 1764
  const int slab_bytes = (slabslots * 16 + 1023) / 1024 * 1024;
  const int ninst = (slabslots + 63) / 64;      // glds wave-instructions per slab
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, gq = lane >> 4;
  const int nwaves = blockDim.x >> 6;
  auto issue = [&](int w, int buf) {
    char* base = smem + buf * slab_bytes;
    for (int j = wave; j < ninst; j += nwaves) {
      const int P = 64 * j + lane;
      if (P < slabslots) {
        const int t = P / rowslots, c = P % rowslots;
        const char* src = qkv + (size_t)token_row(g, w, t) * rowslots * 16 + c * 16;
        __builtin_amdgcn_global_load_lds((gbl_ptr_t)src, (lds_ptr_t)(base + j * 1024), 16, 0, 0);
      }
    }
  };
  // prologue: NBUF-1 windows in flight
  for (int i = 0; i < NBUF - 1; ++i)
    if (w0 + i < w1) issue(w0 + i, i);
  int per_wave = (ninst + nwaves - 1) / nwaves;  // glds per wave per slab (upper bound)
  for (int w = w0, it = 0; w < w1; ++w, ++it) {
    const int buf = it % NBUF;
    if (w + NBUF - 1 < w1) issue(w + NBUF - 1, (it + NBUF - 1) % NBUF);
    // wait for this window's slab: leave the newer NBUF-1 slabs' instructions in flight
    if (w + NBUF - 1 < w1) {
      if (NBUF == 3) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * 10) : "memory");
      else if (NBUF == 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(10) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    (void)per_wave;
    __builtin_amdgcn_s_barrier();
    char* base = smem + buf * slab_bytes;
    // wave = head: read q, k, v fragments
    const int h = wave;
    uint4 q[4], k[4], v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = 16 * i + li < N ? 16 * i + li : 0;
      const char* p = base + (t * rowslots + h * 4 + gq) * 16;
      q[i] = *(const uint4*)p;
      k[i] = *(const uint4*)(p + g.C * 2);
      v[i] = *(const uint4*)(p + g.C * 4);
    }
    float f = fake_math(q[0], D);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (16 * i + li < N) {
        uint4 r = q[i];
        r.x ^= k[i].x ^ v[i].x ^ __float_as_uint(f); r.y ^= k[i].y ^ v[i].y; r.z ^= k[i].z ^ v[i].z; r.w ^= k[i].w ^ v[i].w;
        *(uint4*)(base + ((16 * i + li) * rowslots + h * 4 + gq) * 16) = r;
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // store phase: out rows = q part of the slab rows (C/8 slots per token)
    const int oslots = g.C / 8;
    for (int P = threadIdx.x; P < N * oslots; P += blockDim.x) {
      const int t = P / oslots, c = P % oslots;
      const uint4 r = *(const uint4*)(base + (t * rowslots + c) * 16);
      *(uint4*)(out + (size_t)token_row(g, w, t) * oslots * 16 + c * 16) = r;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
}


// ---- one workgroup per window (non-persistent), full-row staging through LDS
template <bool GLDS, bool NT>
__global__ __launch_bounds__(192) void win1(const char* __restrict__ qkv, char* __restrict__ out, Geom g, int D) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int w = blockIdx.x;
  const int N = g.win * g.win;
  const int rowslots = 3 * g.C / 8, slabslots = N * rowslots;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, gq = lane >> 4;
  const int nwaves = blockDim.x >> 6;
  char* base = smem;
  if (GLDS) {
    for (int j = wave; j * 64 < slabslots; j += nwaves) {
      const int P = 64 * j + lane;
      if (P < slabslots) {
        const int t = P / rowslots, c = P % rowslots;
        const char* src = qkv + (size_t)token_row(g, w, t) * rowslots * 16 + c * 16;
        __builtin_amdgcn_global_load_lds((gbl_ptr_t)src, (lds_ptr_t)(base + j * 1024), 16, 0, NT ? 2 : 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    uint4 r[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      const int P = threadIdx.x + 192 * k;
      if (P < slabslots) {
        const int t = P / rowslots, c = P % rowslots;
        const uint4* src = (const uint4*)(qkv + (size_t)token_row(g, w, t) * rowslots * 16 + c * 16);
        if (NT) {
          typedef unsigned int u4 __attribute__((ext_vector_type(4)));
          r[k] = __builtin_bit_cast(uint4, __builtin_nontemporal_load((const u4*)src));
        } else r[k] = *src;
      }
    }
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      const int P = threadIdx.x + 192 * k;
      if (P < slabslots) *(uint4*)(base + P * 16) = r[k];
    }
  }
  __syncthreads();
  const int h = wave;
  uint4 q[4], k[4], v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int t = 16 * i + li < N ? 16 * i + li : 0;
    const char* p = base + (t * rowslots + h * 4 + gq) * 16;
    q[i] = *(const uint4*)p;
    k[i] = *(const uint4*)(p + g.C * 2);
    v[i] = *(const uint4*)(p + g.C * 4);
  }
  float f = fake_math(q[0], D);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (16 * i + li < N) {
      uint4 r = q[i];
      r.x ^= k[i].x ^ v[i].x ^ __float_as_uint(f); r.y ^= k[i].y ^ v[i].y; r.z ^= k[i].z ^ v[i].z; r.w ^= k[i].w ^ v[i].w;
      *(uint4*)(base + ((16 * i + li) * rowslots + h * 4 + gq) * 16) = r;
    }
  __syncthreads();
  const int oslots = g.C / 8;
  for (int P = threadIdx.x; P < N * oslots; P += blockDim.x) {
    const int t = P / oslots, c = P % oslots;
    const uint4 r = *(const uint4*)(base + (t * rowslots + c) * 16);
    uint4* dst = (uint4*)(out + (size_t)token_row(g, w, t) * oslots * 16 + c * 16);
    if (NT) {
      typedef unsigned int u4 __attribute__((ext_vector_type(4)));
      __builtin_nontemporal_store(__builtin_bit_cast(u4, r), (u4*)dst);
    } else *dst = r;
  }
}

// ---- ideal: same window order, no LDS: each thread moves q,k,v of one (token, 16-B col) -> out
__global__ __launch_bounds__(256) void ideal(const char* __restrict__ qkv, char* __restrict__ out, Geom g) {
  const int oslots = g.C / 8, N = g.win * g.win;
  const long long P = (long long)blockIdx.x * 256 + threadIdx.x;
  if (P >= (long long)g.nwin * N * oslots) return;
  const int w = (int)(P / (N * oslots)), rem = (int)(P % (N * oslots)), t = rem / oslots, c = rem % oslots;
  const int row = token_row(g, w, t);
  const uint4* s = (const uint4*)(qkv + (size_t)row * 3 * oslots * 16) + c;
  uint4 a = s[0], b = s[oslots], d = s[2 * oslots];
  a.x ^= b.x ^ d.x; a.y ^= b.y ^ d.y; a.z ^= b.z ^ d.z; a.w ^= b.w ^ d.w;
  *((uint4*)(out + (size_t)row * oslots * 16) + c) = a;
}

int main(int argc, char** argv) {
  Geom g;
  g.B = 256; g.H = g.W = 56; g.C = 96; g.nH = 3; g.win = 7; g.shift = argc > 1 ? atoi(argv[1]) : 3;
  g.nWh = g.H / g.win; g.nWw = g.W / g.win; g.nwin = g.B * g.nWh * g.nWw;
  const size_t T = (size_t)g.B * g.H * g.W;
  const size_t in_bytes = T * 3 * g.C * 2, out_bytes = T * g.C * 2;
  void *in, *out;
  CK(hipMalloc(&in, in_bytes));
  CK(hipMalloc(&out, out_bytes));
  CK(hipMemset(in, 1, in_bytes));
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
    printf("%-34s %8.1f us  %7.0f GB/s\n", name, ms * 1e3, (in_bytes + out_bytes) / ms / 1e6);
    fflush(stdout);
  };

  {
    const int sl = 49 * 36 * 16;
    const long long tot = (long long)g.nwin * 49 * 12;
    run("ideal (window order, direct)", [&] { hipLaunchKernelGGL(ideal, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, 0, (const char*)in, (char*)out, g); });
    for (int D : {0, 100, 300}) {
      char nm[80];
      snprintf(nm, 80, "win1 reg D=%d", D);
      run(nm, [&] { hipLaunchKernelGGL((win1<false, false>), dim3(g.nwin), dim3(192), sl, 0, (const char*)in, (char*)out, g, D); });
      snprintf(nm, 80, "win1 reg nt D=%d", D);
      run(nm, [&] { hipLaunchKernelGGL((win1<false, true>), dim3(g.nwin), dim3(192), sl, 0, (const char*)in, (char*)out, g, D); });
      snprintf(nm, 80, "win1 glds D=%d", D);
      run(nm, [&] { hipLaunchKernelGGL((win1<true, false>), dim3(g.nwin), dim3(192), 28 * 1024, 0, (const char*)in, (char*)out, g, D); });
      snprintf(nm, 80, "win1 glds nt D=%d", D);
      run(nm, [&] { hipLaunchKernelGGL((win1<true, true>), dim3(g.nwin), dim3(192), 28 * 1024, 0, (const char*)in, (char*)out, g, D); });
    }
  }
  const int slab_bytes = (49 * 36 * 16 + 1023) / 1024 * 1024;
  for (int D : {0, 100, 300}) {
    char nm[80];
    for (int ch : {256 * 4 / 3 / 8 * 8, 1024}) {
      snprintf(nm, 80, "frag chunks=%d D=%d", ch, D);
      run(nm, [&] { hipLaunchKernelGGL(frag, dim3(ch * 3), dim3(256), 0, 0, (const uint4*)in, (uint4*)out, g, ch, D); });
    }
    for (int ch : {256, 512}) {
      snprintf(nm, 80, "slab2 chunks=%d D=%d", ch, D);
      run(nm, [&] { hipLaunchKernelGGL(slab<2>, dim3(ch), dim3(192), 2 * slab_bytes, 0, (const char*)in, (char*)out, g, ch, D); });
      snprintf(nm, 80, "slab3 chunks=%d D=%d", ch, D);
      run(nm, [&] { hipLaunchKernelGGL(slab<3>, dim3(ch), dim3(192), 3 * slab_bytes, 0, (const char*)in, (char*)out, g, ch, D); });
    }
  }
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  return 0;
}
