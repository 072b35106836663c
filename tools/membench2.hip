// Build (not tracked in git): hipcc -O3 --offload-arch=gfx950 tools/membench2.hip -o tools/membench2
// Streaming ceiling for the exact row mix of the edge forward (not part of the library; VERDICT r03
// "reconcile the streaming ceiling"): per edge R streamed 512-B row reads, G gathered 512-B rows from
// two node-sized tables (P / Q: N = E / 6 rows each, the edge forward's P[dst], Q[src], P[src], Q[dst]
// with dst-sorted edges, so the gathers are mostly L2 hits) and W streamed 512-B row writes.
//
// Persistent blocks own contiguous row ranges and walk them in 32-row rounds (the edge kernels'
// layout: whole-row access, 16 B per lane, a wave instruction covers 2 rows); the loads of DEPTH
// rounds are in flight (a register ring, the next round's gathers issued a round ahead when
// DEPTH > 1); stores default or nontemporal.  Swept: DEPTH 1..3, 8 or 16 waves per CU (1 or 2
// blocks of 512 threads), default / nt stores, the edge forward's 2R + 4G + 5W and its parts.  A
// grid-stride float4 copy over 1 GiB arrays (the guide's "float4 copy", MI355X_MICROARCH.md:36)
// anchors the table.  No compute: this is the memory system's rate for the shape, the floor under
// the kernel.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/membench2 tools/membench2.hip && tools/membench2
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int L = 128;
constexpr int ROUND = 32;
constexpr int THREADS = 512;
constexpr int U = ROUND * 32 / THREADS;   // row slots per thread per round (2)

__device__ __forceinline__ int clampr(int r, int r1) { return r < r1 ? r : r1 - 1; }

// XI: XCD-interleaved rounds (blocks b and b + 8 share an XCD's L2: each XCD owns a contiguous eighth of
// the rows and its blocks take its 32-row rounds round-robin, so the XCD's blocks sweep its range
// together and the gathered rows' reuse stays inside its L2); otherwise one contiguous range per block.
template <int R, int G, int W, int DEPTH, bool NT, int BPC, bool XI = false, bool IL = false, int GSEL = 0>
__global__ __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(2 * BPC, 2 * BPC))) void mix(const float* const* __restrict__ in, float* const* __restrict__ out,
                                               const int* __restrict__ gd, const int* __restrict__ gs,
                                               const float* __restrict__ P, const float* __restrict__ Q, int E) {
  const int nb = gridDim.x;
  int r0, r1, step;
  if (XI) {
    const int rounds = (E + ROUND - 1) / ROUND, perx = (rounds + 7) / 8;
    const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
    r0 = min(E, (x * perx + j) * ROUND);
    r1 = min(E, (x + 1) * perx * ROUND);
    step = (nb >> 3) * ROUND;
  } else {
    int per = (E + nb - 1) / nb;
    per = (per + ROUND - 1) / ROUND * ROUND;
    r0 = min(E, per * (int)blockIdx.x);
    r1 = min(E, per * ((int)blockIdx.x + 1));
    step = ROUND;
  }
  if (r0 >= r1) return;
  const int t = threadIdx.x, c = 4 * (t & 31), rr = t >> 5;
  constexpr int RG = R > 0 ? R : 1;
  constexpr int GG = G > 0 ? G : 1;
  f32x4 v[DEPTH][RG][U];
  int di[DEPTH][U], si[DEPTH][U];
  f32x4 g[DEPTH][GG][U];
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  auto issue = [&](int s, int base) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = clampr(base + rr + 16 * u, min(r1, max(base, 0) + ROUND));
#pragma unroll
      for (int a = 0; a < R; ++a) v[s][a][u] = *reinterpret_cast<const f32x4*>(in[a] + (size_t)row * L + c);
      if (G) {
        di[s][u] = gd[row];
        si[s][u] = gs[row];
      }
    }
  };
  auto gather = [&](int gslot, int s) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int a = 0; a < G; ++a) {
        // GSEL 1: only the source-side rows (Q[src], P[src]) of the four, 2: only the destination-side ones
        const bool src_side = (a >> 1) ^ (a & 1);
        if ((GSEL == 1 && !src_side) || (GSEL == 2 && src_side)) {
          g[gslot][a][u] = f32x4{0.f, 0.f, 0.f, 0.f};
          continue;
        }
        const int node = src_side ? si[s][u] : di[s][u];
        // IL: P and Q interleaved per node ([P | Q], 1 KB rows in P's buffer): a node's two rows adjacent
        const float* row = IL ? P + (size_t)node * 2 * L + ((a & 1) ? L : 0) : ((a & 1) ? Q : P) + (size_t)node * L;
        g[gslot][a][u] = *reinterpret_cast<const f32x4*>(row + c);
      }
  };
#pragma unroll
  for (int s = 0; s < DEPTH; ++s) issue(s, r0 + step * s);
  if (G && DEPTH > 1) gather(0, 0);
  for (int base = r0; base < r1; base += DEPTH * step) {
#pragma unroll
    for (int s = 0; s < DEPTH; ++s) {
      const int b = base + step * s;
      // DEPTH > 1: round b's gathers were issued a round ahead (slot s); the next round's now
      if (G && DEPTH == 1) gather(0, 0);
      if (G && DEPTH > 1) gather((s + 1) % DEPTH, (s + 1) % DEPTH);
      f32x4 x = acc;
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int a = 0; a < R; ++a) x += v[s][a][u];
#pragma unroll
        for (int a = 0; a < G; ++a) x += g[s][a][u];
      }
      acc = x;
      issue(s, b + DEPTH * step);   // clamped past r1
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int row = clampr(b + rr + 16 * u, min(r1, b + ROUND));
#pragma unroll
        for (int a = 0; a < W; ++a) {
          f32x4* p = reinterpret_cast<f32x4*>(out[a] + (size_t)row * L + c);
          const f32x4 y = x + (float)a;
          if (NT) __builtin_nontemporal_store(y, p);
          else *p = y;
        }
      }
    }
  }
  if (W == 0 && acc[0] == 123.456f) out[0][0] = acc[1];   // keep the loads live
}

// SPLIT: the same rows and bytes as mix<2, 4, 5, 1, true>, but waves 0-3 only stream (2 reads, 5 nt writes
// of each row) and waves 4-7 only gather (the 4 P / Q rows of each edge, summed into a register): is the
// gathers' cost their own, or the streams' waits behind them in the same waves?
__global__ __launch_bounds__(THREADS) void split_mix(const float* const* __restrict__ in, float* const* __restrict__ out,
                                                     const int* __restrict__ gd, const int* __restrict__ gs,
                                                     const float* __restrict__ P, const float* __restrict__ Q, int E) {
  const int nb = gridDim.x;
  int per = (E + nb - 1) / nb;
  per = (per + ROUND - 1) / ROUND * ROUND;
  const int r0 = min(E, per * (int)blockIdx.x), r1 = min(E, per * ((int)blockIdx.x + 1));
  if (r0 >= r1) return;
  const int t = threadIdx.x & 255, c = 4 * (t & 31), rr = t >> 5;   // 8 rows per instruction, 4 slots
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (threadIdx.x < 256) {
    f32x4 v[2][4];
    auto issue = [&](int base) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int row = clampr(base + rr + 8 * u, r1);
#pragma unroll
        for (int a = 0; a < 2; ++a) v[a][u] = *reinterpret_cast<const f32x4*>(in[a] + (size_t)row * L + c);
      }
    };
    issue(r0);
    for (int base = r0; base < r1; base += ROUND) {
      f32x4 x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) x[u] = v[0][u] + v[1][u];
      issue(base + ROUND);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int row = clampr(base + rr + 8 * u, r1);
#pragma unroll
        for (int a = 0; a < 5; ++a)
          __builtin_nontemporal_store(x[u] + (float)a, reinterpret_cast<f32x4*>(out[a] + (size_t)row * L + c));
      }
    }
  } else {
    int di[4], si[4];
    f32x4 g[4][4];
    auto ids = [&](int base) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int row = clampr(base + rr + 8 * u, r1);
        di[u] = gd[row];
        si[u] = gs[row];
      }
    };
    ids(r0);
    for (int base = r0; base < r1; base += ROUND) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        g[0][u] = *reinterpret_cast<const f32x4*>(P + (size_t)di[u] * L + c);
        g[1][u] = *reinterpret_cast<const f32x4*>(Q + (size_t)si[u] * L + c);
        g[2][u] = *reinterpret_cast<const f32x4*>(P + (size_t)si[u] * L + c);
        g[3][u] = *reinterpret_cast<const f32x4*>(Q + (size_t)di[u] * L + c);
      }
      ids(base + ROUND);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc += (g[0][u] + g[1][u]) + (g[2][u] + g[3][u]);
    }
    if (acc[0] == 123.456f) out[0][0] = acc[1];
  }
}

__global__ void copy4(const f32x4* __restrict__ a, f32x4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

struct Bufs {
  float** d_in;
  float** d_out;
  int* gd;
  int* gs;
  int* gd_small;   // the same pattern folded onto 1,024 nodes (1 MB of P / Q rows: surely L2-resident)
  int* gs_small;
  float* P;
  float* Q;
  int E;
  int N;
};

template <typename F>
double time_us(F launch, int reps = 20) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) launch();
  (void)hipEventRecord(a);
  for (int i = 0; i < reps; ++i) launch();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return ms * 1e3 / reps;
}

template <int R, int G, int W, int DEPTH, bool NT, int BPC = 1, bool XI = false, bool IL = false, int GSEL = 0>
void run(const Bufs& B, int cus, bool small = false) {
  const int blocks_per_cu = BPC;
  const int nblk = cus * blocks_per_cu;
  const double us = time_us([&] {
    hipLaunchKernelGGL((mix<R, G, W, DEPTH, NT, BPC, XI, IL, GSEL>), dim3(nblk), dim3(THREADS), 0, 0, B.d_in, B.d_out,
                       small ? B.gd_small : B.gd, small ? B.gs_small : B.gs, B.P, B.Q, B.E);
  });
  const double streamed = (double)B.E * 512.0 * (R + W);
  const double gathered = (double)B.E * 512.0 * G;
  printf("{\"mix\": \"%dR+%dG+%dW\", \"table\": \"%s%s\", \"rows\": \"%s\", \"depth\": %d, \"waves_per_cu\": %d, \"stores\": \"%s\", \"us\": %.1f, "
         "\"streamed_TBps\": %.3f, \"with_gathers_TBps\": %.3f}\n",
         R, G, W, small ? "1k nodes" : "N nodes", IL ? ", P|Q interleaved" : (GSEL == 1 ? ", src-side gathers only" : (GSEL == 2 ? ", dst-side gathers only" : "")), XI ? "xcd-interleaved" : "contiguous", DEPTH, 8 * blocks_per_cu, NT ? "nt" : "default", us, streamed / us * 1e-6,
         (streamed + gathered) / us * 1e-6);
  fflush(stdout);
}

int main() {
  const int E = 239744;   // config 2's edges
  const int N = 40328;    // config 2's nodes
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  std::vector<float*> bufs(14);
  for (auto& p : bufs) {
    (void)hipMalloc(&p, (size_t)E * 512);
    (void)hipMemset(p, 0, (size_t)E * 512);
  }
  Bufs B{};
  B.E = E;
  B.N = N;
  (void)hipMalloc(&B.d_in, 7 * sizeof(float*));
  (void)hipMalloc(&B.d_out, 7 * sizeof(float*));
  (void)hipMemcpy(B.d_in, bufs.data(), 7 * sizeof(float*), hipMemcpyHostToDevice);
  (void)hipMemcpy(B.d_out, bufs.data() + 7, 7 * sizeof(float*), hipMemcpyHostToDevice);
  // dst-sorted edges of a periodic 71 x 71-like mesh: ~6 per node, sources at mesh-neighbour offsets
  std::vector<int> hd(E), hs(E);
  const int offs[6] = {1, -1, 71, -71, 72, -72};
  for (int e = 0; e < E; ++e) {
    hd[e] = (int)((long long)e * N / E);
    hs[e] = ((hd[e] + offs[e % 6]) % N + N) % N;
  }
  (void)hipMalloc(&B.gd, E * sizeof(int));
  (void)hipMalloc(&B.gs, E * sizeof(int));
  (void)hipMemcpy(B.gd, hd.data(), E * sizeof(int), hipMemcpyHostToDevice);
  (void)hipMemcpy(B.gs, hs.data(), E * sizeof(int), hipMemcpyHostToDevice);
  for (int e = 0; e < E; ++e) {
    hd[e] &= 1023;
    hs[e] &= 1023;
  }
  (void)hipMalloc(&B.gd_small, E * sizeof(int));
  (void)hipMalloc(&B.gs_small, E * sizeof(int));
  (void)hipMemcpy(B.gd_small, hd.data(), E * sizeof(int), hipMemcpyHostToDevice);
  (void)hipMemcpy(B.gs_small, hs.data(), E * sizeof(int), hipMemcpyHostToDevice);
  (void)hipMalloc(&B.P, (size_t)N * 1024);   // room for the interleaved [P | Q] table
  (void)hipMalloc(&B.Q, (size_t)N * 512);
  (void)hipMemset(B.P, 0, (size_t)N * 1024);
  (void)hipMemset(B.Q, 0, (size_t)N * 512);

  {  // the guide's anchor: grid-stride float4 copy over 1 GiB arrays
    const size_t n = (size_t)1 << 26;   // f32x4 elements = 1 GiB
    f32x4 *a, *b;
    (void)hipMalloc(&a, n * 16);
    (void)hipMalloc(&b, n * 16);
    (void)hipMemset(a, 0, n * 16);
    (void)hipMemset(b, 0, n * 16);
    const double us = time_us([&] { hipLaunchKernelGGL(copy4, dim3(cus * 16), dim3(256), 0, 0, a, b, n); }, 10);
    printf("{\"mix\": \"copy 1 GiB float4 grid-stride\", \"us\": %.1f, \"streamed_TBps\": %.3f}\n", us,
           2.0 * n * 16 / us * 1e-6);
    (void)hipFree(a);
    (void)hipFree(b);
  }
  // P / Q as two tables vs interleaved per node, contiguous and XCD-interleaved rows (the edge forward's)
  if (getenv("MB_EBW")) {   // the edge backward's mixes: the split pair today vs a fused pass (memory only)
    for (int rep = 0; rep < 3; ++rep) {
      run<5, 1, 2, 2, false>(B, cus);   // edge_bwd_w2: gaggr[dst] + a2m, a1m, ge_next, a2e, a1e -> gz1m, gC
      run<4, 0, 1, 2, false>(B, cus);   // edge_gout_wc: gC, e, ge_next, a2ln -> ge_out
      run<7, 1, 3, 2, false>(B, cus);   // fused: + e, a2ln; -> gz1m, gC, ge_out (no gC re-read, one ge_next)
    }
    return 0;
  }
  if (getenv("MB_GSEL")) {   // which half of the four gathers costs what beside the streams
    for (int rep = 0; rep < 3; ++rep) {
      run<2, 4, 5, 1, true, 1, true, false, 0>(B, cus);
      run<2, 4, 5, 1, true, 1, true, false, 1>(B, cus);
      run<2, 4, 5, 1, true, 1, true, false, 2>(B, cus);
      run<2, 0, 5, 1, true, 1, true>(B, cus);
    }
    return 0;
  }
  if (getenv("MB_IL")) {
    for (int rep = 0; rep < 3; ++rep) {
      run<2, 4, 5, 1, true, 1, false, false>(B, cus);
      run<2, 4, 5, 1, true, 1, false, true>(B, cus);
      run<2, 4, 5, 1, true, 1, true, false>(B, cus);
      run<2, 4, 5, 1, true, 1, true, true>(B, cus);
      run<0, 4, 0, 1, true, 1, true, false>(B, cus);
      run<0, 4, 0, 1, true, 1, true, true>(B, cus);
    }
    return 0;
  }
  // the edge forward's mix in one set of waves vs split over stream waves and gather waves
  for (int rep = 0; rep < 2; ++rep) {
    run<2, 4, 5, 1, true>(B, cus);
    run<2, 0, 5, 1, true>(B, cus);
    run<0, 4, 0, 1, true>(B, cus);
    const double us = time_us([&] {
      hipLaunchKernelGGL(split_mix, dim3(cus), dim3(THREADS), 0, 0, B.d_in, B.d_out, B.gd, B.gs, B.P, B.Q, B.E);
    });
    printf("{\"mix\": \"2R+4G+5W split waves (0-3 stream, 4-7 gather)\", \"us\": %.1f, \"streamed_TBps\": %.3f}\n", us,
           (double)B.E * 512.0 * 7 / us * 1e-6);
    fflush(stdout);
  }
  return 0;
}
