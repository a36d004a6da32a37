// Memory-shape probe for the W-MSA BACKWARD at the SwinV2-T stage-0 shape (T = 256*56*56,
// C = 96, 3 heads, window 7, shift 3): the backward's bytes (read qkv [T,3C] and dO [T,C],
// write dqkv [T,3C], bf16 -- 14 C bytes per token) moved with no attention math, in the
// access shapes a kernel could use:
//   pair  - wmsa_bwd_pair_kernel's shape: a (window, head) per wave pair, 16 token rows x 64 B
//           per 16-B-per-lane instruction (own q/k/dO tiles + all V tiles per wave), 2 pairs
//           per 4-wave workgroup, 2 workgroups per CU
//   slab  - one workgroup per window chunk, ALL heads: each token's whole qkv row (3C) and
//           dO row (C) read and its whole dqkv row written, as the window's 7 row runs of
//           7 tokens (contiguous 4 KB runs of qkv at stage 0)
//   lin   - the same bytes as one linear stream (the ceiling)
// Optional fake VALU work D per (window, head) emulates the math.
//   hipcc --offload-arch=gfx950 -O3 wmsa_bwd_mem.hip -o wmsa_bwd_mem && ./wmsa_bwd_mem
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(err_)); return 1; } } while (0)

struct Geom { int B, H, W, C, nH, win, shift, nWh, nWw, nwin; };

__device__ __forceinline__ int token_row(const Geom& g, int w, int t) {
  const int per = g.nWh * g.nWw;
  const int b = w / per, rem = w % per, wh = rem / g.nWw, ww = rem % g.nWw;
  int y = wh * g.win + t / g.win + g.shift, x = ww * g.win + t % g.win + g.shift;
  if (y >= g.H) y -= g.H;
  if (x >= g.W) x -= g.W;
  return (b * g.H + y) * g.W + x;
}

__device__ __forceinline__ uint4 mix(uint4 a, uint4 b, int D) {
  uint4 r = make_uint4(a.x ^ b.y, a.y ^ b.x, a.z + b.w, a.w - b.z);
  for (int i = 0; i < D; ++i) r = make_uint4(r.x * 3 + r.y, r.y ^ r.z, r.z + r.w, r.w * 5 + r.x);
  return r;
}

// ---- pair: wmsa_bwd_pair_kernel's per-lane access shape
__global__ __launch_bounds__(256, 2) void pair(const uint4* __restrict__ qkv, const uint4* __restrict__ dout,
                                               uint4* __restrict__ dqkv, Geom g, int chunks, int D) {
  const int h = blockIdx.x % g.nH, chunk = blockIdx.x / g.nH;
  const int w0 = (int)((long long)chunk * g.nwin / chunks), w1 = (int)((long long)(chunk + 1) * g.nwin / chunks);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int pr = wave >> 1, hf = wave & 1, li = lane & 15, gq = lane >> 4;
  const int C3u = 3 * g.C / 8, Cu = g.C / 8, hu = h * 4 + gq;
  for (int w = w0 + pr; w < w1; w += 2) {
    uint4 v[4], q[2], k[2], d[2];
    int row[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int tok = 16 * t + li;
      row[t] = token_row(g, w, tok < 49 ? tok : 0);
      v[t] = tok < 49 ? qkv[(size_t)row[t] * C3u + 2 * Cu + hu] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int t = hf + 2 * j, tok = 16 * t + li;
      const int r = hf ? row[2 * j + 1] : row[2 * j];
      if (tok < 49) {
        q[j] = qkv[(size_t)r * C3u + hu];
        k[j] = qkv[(size_t)r * C3u + Cu + hu];
        d[j] = dout[(size_t)r * Cu + hu];
      } else {
        q[j] = k[j] = d[j] = make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int t = hf + 2 * j, tok = 16 * t + li;
      const int r = hf ? row[2 * j + 1] : row[2 * j];
      if (tok < 49) {
        dqkv[(size_t)r * C3u + hu] = mix(q[j], d[j], D);
        dqkv[(size_t)r * C3u + Cu + hu] = mix(k[j], v[2 * j], D);
        dqkv[(size_t)r * C3u + 2 * Cu + hu] = mix(v[2 * j + 1], d[j], D);
      }
    }
  }
}

// ---- slab: one workgroup per window chunk, all heads; per window the 49 tokens' whole rows
// as 16-B units: qkv row = 3C/8 units, dO row = C/8 units.  Lane-consecutive units of one
// row run are contiguous in memory (7 tokens of a window row are adjacent tokens).
__global__ __launch_bounds__(256, 2) void slab(const uint4* __restrict__ qkv, const uint4* __restrict__ dout,
                                               uint4* __restrict__ dqkv, Geom g, int chunks, int D) {
  const int chunk = blockIdx.x;
  const int w0 = (int)((long long)chunk * g.nwin / chunks), w1 = (int)((long long)(chunk + 1) * g.nwin / chunks);
  const int C3u = 3 * g.C / 8, Cu = g.C / 8;
  const int per_win = 49 * C3u;  // qkv units per window
  for (int w = w0; w < w1; ++w) {
    for (int e = threadIdx.x; e < per_win; e += 256) {
      const int tok = e / C3u, u = e % C3u;
      const size_t r = token_row(g, w, tok);
      const uint4 x = qkv[r * C3u + u];
      const uint4 dd = dout[r * Cu + (u % Cu)];
      dqkv[r * C3u + u] = mix(x, dd, D);
    }
  }
}

// ---- grp: one workgroup per (window chunk, head pair): each token's 128-B pieces of q, k, v
// and dO for the pair read as contiguous 16-B units; FRAG = 0 writes dq/dk/dv as the same
// 128-B pieces, FRAG = 1 as the kernels do (16 token rows x 64 B per instruction per head)
template <int FRAG>
__global__ __launch_bounds__(256, 2) void grp(const uint4* __restrict__ qkv, const uint4* __restrict__ dout,
                                              uint4* __restrict__ dqkv, Geom g, int chunks, int D) {
  const int ng = g.nH / 2;
  const int gr = blockIdx.x % ng, chunk = blockIdx.x / ng;
  const int w0 = (int)((long long)chunk * g.nwin / chunks), w1 = (int)((long long)(chunk + 1) * g.nwin / chunks);
  const int C3u = 3 * g.C / 8, Cu = g.C / 8, go = gr * 8;  // 16-B units
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int w = w0; w < w1; ++w) {
    // 49 tokens x (3 parts + dO) x 8 units
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (int e = threadIdx.x; e < 49 * 32; e += 256) {
      const int tok = e >> 5, part = (e >> 3) & 3, u = e & 7;
      const size_t r = token_row(g, w, tok);
      const uint4 x = part < 3 ? qkv[r * C3u + part * Cu + go + u] : dout[r * Cu + go + u];
      acc = mix(acc, x, D);
      if (!FRAG && part < 3) dqkv[r * C3u + part * Cu + go + u] = acc;
    }
    if (FRAG) {
      // 2 heads x 3 parts x 4 tiles of (16 rows x 64 B): one per wave-instruction
      const int li = lane & 15, gq = lane >> 4;
      for (int k = wave; k < 24; k += 4) {
        const int hh = k / 12, part = (k / 4) % 3, t = k % 4;
        const int tok = 16 * t + li;
        if (tok < 49) {
          const size_t r = token_row(g, w, tok);
          dqkv[r * C3u + part * Cu + go + 4 * hh + gq] = acc;
        }
      }
    }
  }
}

// ---- lin: the same bytes as a linear stream
__global__ __launch_bounds__(256) void lin(const uint4* __restrict__ qkv, const uint4* __restrict__ dout,
                                           uint4* __restrict__ dqkv, size_t n3, int Cu, int C3u) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n3; i += (size_t)gridDim.x * 256) {
    const size_t r = i / C3u, u = i % C3u;
    dqkv[i] = mix(qkv[i], dout[r * Cu + (u % Cu)], 0);
  }
}

int main(int argc, char** argv) {
  Geom g;
  g.B = 256; g.H = 56; g.W = 56; g.C = 96; g.nH = 3; g.win = 7; g.shift = 3;
  if (argc > 1 && atoi(argv[1]) == 2) { g.H = g.W = 14; g.C = 384; g.nH = 12; }  // stage 2
  if (argc > 1 && atoi(argv[1]) == 1) { g.H = g.W = 28; g.C = 192; g.nH = 6; }   // stage 1
  g.nWh = g.H / g.win; g.nWw = g.W / g.win; g.nwin = g.B * g.nWh * g.nWw;
  const size_t T = (size_t)g.B * g.H * g.W;
  const size_t qkv_b = T * 3 * g.C * 2, do_b = T * g.C * 2;
  uint4 *qkv, *dout, *dqkv;
  CK(hipMalloc(&qkv, qkv_b)); CK(hipMalloc(&dout, do_b)); CK(hipMalloc(&dqkv, qkv_b));
  CK(hipMemset(qkv, 1, qkv_b)); CK(hipMemset(dout, 2, do_b)); CK(hipMemset(dqkv, 0, qkv_b));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const double bytes = 2.0 * qkv_b + do_b;
  auto run = [&](const char* name, auto launch) -> int {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    const int it = 20;
    for (int i = 0; i < it; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= it;
    printf("%-30s %8.1f us  %7.0f GB/s\n", name, ms * 1e3, bytes / ms / 1e6);
    return 0;
  };
  char nm[80];
  run("lin", [&] { hipLaunchKernelGGL(lin, dim3(4096), dim3(256), 0, 0, qkv, dout, dqkv, T * 3 * g.C / 8, g.C / 8, 3 * g.C / 8); });
  for (int D : {0, 64}) {
    const int chunks = 512 / g.nH;
    snprintf(nm, 80, "pair chunks=%d D=%d", chunks, D);
    run(nm, [&] { hipLaunchKernelGGL(pair, dim3(chunks * g.nH), dim3(256), 0, 0, qkv, dout, dqkv, g, chunks, D); });
    for (int ch : {256 / (g.nH / 2) * 2, 512 / (g.nH / 2)}) {
      snprintf(nm, 80, "grp128 store-128B chunks=%d D=%d", ch, D);
      run(nm, [&] { hipLaunchKernelGGL(grp<0>, dim3(ch * (g.nH / 2)), dim3(256), 0, 0, qkv, dout, dqkv, g, ch, D); });
      snprintf(nm, 80, "grp128 store-frag chunks=%d D=%d", ch, D);
      run(nm, [&] { hipLaunchKernelGGL(grp<1>, dim3(ch * (g.nH / 2)), dim3(256), 0, 0, qkv, dout, dqkv, g, ch, D); });
    }
    for (int ch : {512, 1024, 2048}) {
      snprintf(nm, 80, "slab chunks=%d D=%d", ch, D);
      run(nm, [&] { hipLaunchKernelGGL(slab, dim3(ch), dim3(256), 0, 0, qkv, dout, dqkv, g, ch, D); });
    }
  }
  return 0;
}
