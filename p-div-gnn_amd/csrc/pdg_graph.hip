// Mesh graph construction on the device: the "with preprocessing"
// path of the reference (benchmark_gnn_fem.py:388-415, datasets.py:247-263):
//   mesh_to_graph     (convert_utils.py:47-60, PyG FaceToEdge: the 3 edges of every
//                      triangle in both directions, coalesced),
//   edge lengths      (datasets.py:182-188, |pos[row] - pos[col]| over all coordinates),
//   compute_periodic_graph (datasets.py:39-119: left<->right and lower<->upper side nodes
//                      paired in (y, x) order, the 4 corners paired with the opposite
//                      corner, zero edge attribute for the new edges, coalesced with
//                      sum-reduced attributes).
//
// No global sort: the result is a per-row (CSR) object.  Directed edges are counted per
// source row, scattered into the rows' slots in any order (atomics), every row is sorted
// and de-duplicated by itself (rows are short), and a prefix sum places the unique edges.
// The sorted-within-row, rows-in-order result is exactly PyG's coalesce order (by
// row * N + col).  A coalesced attribute is the sum over duplicates of (length for a mesh
// edge, 0 for a periodic one) = the length if the pair is a mesh edge, else 0, so the
// length is computed once per unique edge.  Everything is integer-exact and independent
// of the atomics' order; the lengths are fp32 in torch.linalg.vector_norm's CPU order
// (s = dx*dx, s = fma(dy, dy, s) [, fma(dz, dz, s)], correctly rounded sqrt: bitwise equal).
//
// The side lists are sorted by one workgroup (bitonic, in LDS): each side holds at most
// PDG_SIDE_MAX nodes (a 4096 x 4096 grid).  Invalid periodic geometry (unequal opposite
// sides, a corner that is not exactly one node, a side longer than PDG_SIDE_MAX) is
// reported as *n_edges = -1.
#include <cfloat>

#include "pdg_common.hpp"
#include "pdg_runtime.hpp"

#ifndef PDG_SIDE_MAX
#define PDG_SIDE_MAX 4096
#endif

using namespace pdg;

namespace {

constexpr int GT = 256;                  // threads per block of the elementwise kernels
constexpr int SIDE_MAX = PDG_SIDE_MAX;   // nodes per periodic side
constexpr int SORT_THREADS = 1024;

// Scratch layout (int32 words unless noted), see pdg_mesh_graph_scratch_bytes.
struct Scratch {
  float* bbox;     // [GT_BLOCKS_MAX][4] per-block (min x, min y, max x, max y)
  int* ctr;        // [16]: side counts (4), corner counts (4), corners (4), npairs, error
  int* side;       // [4][SIDE_MAX]
  int* prow;       // [2 * 2 * SIDE_MAX + 4]
  int* pcol;
  int* deg;        // [N + 1] -> exclusive offsets
  int* fill;       // [N]
  int* ucnt;       // [N + 1] -> row pointer of the result
  int* bsum;       // [scan blocks + 1]
  int* nb;         // [6F + pairs] slot array: 2 * col + (1 if periodic else 0)
};

constexpr int BBOX_BLOCKS = 256;
constexpr int SCAN_BLOCK = 1024;         // elements per scan block (256 threads x 4)

__device__ __forceinline__ float nmul(float a, float b) { return __fmul_rn(a, b); }

__global__ __launch_bounds__(GT) void bbox_kernel(int n, const float* __restrict__ p, int dim, float* __restrict__ part,
                                                  int* __restrict__ ctr) {
  __shared__ float red[4][GT];
  float mnx = FLT_MAX, mny = FLT_MAX, mxx = -FLT_MAX, mxy = -FLT_MAX;
  for (int i = blockIdx.x * GT + threadIdx.x; i < n; i += gridDim.x * GT) {
    const float x = p[(size_t)i * dim], y = p[(size_t)i * dim + 1];
    mnx = fminf(mnx, x);
    mny = fminf(mny, y);
    mxx = fmaxf(mxx, x);
    mxy = fmaxf(mxy, y);
  }
  red[0][threadIdx.x] = mnx;
  red[1][threadIdx.x] = mny;
  red[2][threadIdx.x] = mxx;
  red[3][threadIdx.x] = mxy;
  __syncthreads();
  for (int s = GT / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      red[0][threadIdx.x] = fminf(red[0][threadIdx.x], red[0][threadIdx.x + s]);
      red[1][threadIdx.x] = fminf(red[1][threadIdx.x], red[1][threadIdx.x + s]);
      red[2][threadIdx.x] = fmaxf(red[2][threadIdx.x], red[2][threadIdx.x + s]);
      red[3][threadIdx.x] = fmaxf(red[3][threadIdx.x], red[3][threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x < 4) part[4 * blockIdx.x + threadIdx.x] = red[threadIdx.x][0];
  if (blockIdx.x == 0 && threadIdx.x < 16) ctr[threadIdx.x] = 0;
}

// Side membership (exact float equality, as the reference's ==), compaction into the 4
// side lists (left, right, lower, upper: the concatenation order of datasets.py:85-100)
// and the 4 corners (left-lower, left-upper, right-lower, right-upper).
__global__ __launch_bounds__(GT) void sides_kernel(int n, const float* __restrict__ p, int dim,
                                                   const float* __restrict__ part, int nparts, int* __restrict__ ctr,
                                                   int* __restrict__ side) {
  __shared__ float bb[4];
  if (threadIdx.x < 4) {
    float v = part[threadIdx.x];
    for (int b = 1; b < nparts; ++b) v = threadIdx.x < 2 ? fminf(v, part[4 * b + threadIdx.x]) : fmaxf(v, part[4 * b + threadIdx.x]);
    bb[threadIdx.x] = v;
  }
  __syncthreads();
  const float mnx = bb[0], mny = bb[1], mxx = bb[2], mxy = bb[3];
  for (int i = blockIdx.x * GT + threadIdx.x; i < n; i += gridDim.x * GT) {
    const float x = p[(size_t)i * dim], y = p[(size_t)i * dim + 1];
    const bool on[4] = {x == mnx, x == mxx, y == mny, y == mxy};
#pragma unroll
    for (int s = 0; s < 4; ++s)
      if (on[s]) {
        const int k = atomicAdd(&ctr[s], 1);
        if (k < SIDE_MAX) side[s * SIDE_MAX + k] = i;
      }
    const int c = on[0] && on[2] ? 0 : on[0] && on[3] ? 1 : on[1] && on[2] ? 2 : on[1] && on[3] ? 3 : -1;
    if (c >= 0) {
      atomicAdd(&ctr[4 + c], 1);
      ctr[8 + c] = i;   // meaningful only when the count is exactly 1
    }
  }
}

// One workgroup: sort each side by (y, x, node id) -- np.lexsort((x, y)) is stable, so equal
// (y, x) keep node order -- validate, and emit the periodic pairs in the reference's order.
__global__ __launch_bounds__(SORT_THREADS) void pairs_kernel(const float* __restrict__ p, int dim, int* __restrict__ ctr,
                                                             int* __restrict__ side, int* __restrict__ prow,
                                                             int* __restrict__ pcol) {
  __shared__ float ky[SIDE_MAX], kx[SIDE_MAX];
  __shared__ int ki[SIDE_MAX];
  __shared__ int bad;
  if (threadIdx.x == 0) {
    bad = 0;
    for (int s = 0; s < 4; ++s) bad |= ctr[s] > SIDE_MAX || ctr[s] == 0;
    for (int c = 0; c < 4; ++c) bad |= ctr[4 + c] != 1;
    bad |= ctr[0] != ctr[1] || ctr[2] != ctr[3];
  }
  __syncthreads();
  if (bad) {
    if (threadIdx.x == 0) ctr[13] = 1;
    return;
  }
  for (int s = 0; s < 4; ++s) {
    const int c = ctr[s];
    int np2 = 1;
    while (np2 < c) np2 <<= 1;
    for (int i = threadIdx.x; i < np2; i += blockDim.x) {
      if (i < c) {
        const int v = side[s * SIDE_MAX + i];
        ky[i] = p[(size_t)v * dim + 1];
        kx[i] = p[(size_t)v * dim];
        ki[i] = v;
      } else {
        ky[i] = FLT_MAX;
        kx[i] = FLT_MAX;
        ki[i] = 0x7fffffff;
      }
    }
    __syncthreads();
    for (int k = 2; k <= np2; k <<= 1)
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = threadIdx.x; i < np2; i += blockDim.x) {
          const int o = i ^ j;
          if (o > i) {
            const bool asc = (i & k) == 0;
            const bool gt = ky[i] > ky[o] || (ky[i] == ky[o] && (kx[i] > kx[o] || (kx[i] == kx[o] && ki[i] > ki[o])));
            if (gt == asc) {
              float t = ky[i]; ky[i] = ky[o]; ky[o] = t;
              t = kx[i]; kx[i] = kx[o]; kx[o] = t;
              const int u = ki[i]; ki[i] = ki[o]; ki[o] = u;
            }
          }
        }
        __syncthreads();
      }
    for (int i = threadIdx.x; i < c; i += blockDim.x) side[s * SIDE_MAX + i] = ki[i];
    __syncthreads();
  }
  // rows = [left, right, lower, upper, corners], cols = [right, left, upper, lower, corners reversed]
  const int nl = ctr[0], nd = ctr[2];
  const int* L0 = side;
  const int* R0 = side + SIDE_MAX;
  const int* D0 = side + 2 * SIDE_MAX;
  const int* U0 = side + 3 * SIDE_MAX;
  for (int i = threadIdx.x; i < nl; i += blockDim.x) {
    prow[i] = L0[i];
    pcol[i] = R0[i];
    prow[nl + i] = R0[i];
    pcol[nl + i] = L0[i];
  }
  for (int i = threadIdx.x; i < nd; i += blockDim.x) {
    prow[2 * nl + i] = D0[i];
    pcol[2 * nl + i] = U0[i];
    prow[2 * nl + nd + i] = U0[i];
    pcol[2 * nl + nd + i] = D0[i];
  }
  if (threadIdx.x < 4) {
    prow[2 * nl + 2 * nd + threadIdx.x] = ctr[8 + threadIdx.x];
    pcol[2 * nl + 2 * nd + threadIdx.x] = ctr[8 + 3 - threadIdx.x];
  }
  if (threadIdx.x == 0) ctr[12] = 2 * nl + 2 * nd + 4;
}

// Directed edges of face f: (a,b) (b,a) (b,c) (c,b) (a,c) (c,a) -- FaceToEdge's three edges,
// made undirected.  Pairs k: (prow[k], pcol[k]).
__device__ __forceinline__ void face_edge(const int64_t* __restrict__ faces, int f, int j, int& u, int& v) {
  const int64_t* t = faces + 3 * (size_t)f;
  const int a = (int)t[0], b = (int)t[1], c = (int)t[2];
  switch (j) {
    case 0: u = a; v = b; break;
    case 1: u = b; v = a; break;
    case 2: u = b; v = c; break;
    case 3: u = c; v = b; break;
    case 4: u = a; v = c; break;
    default: u = c; v = a; break;
  }
}

__global__ __launch_bounds__(GT) void count_kernel(int n, int nf, const int64_t* __restrict__ faces,
                                                   const int* __restrict__ ctr, const int* __restrict__ prow,
                                                   int* __restrict__ deg, int* __restrict__ fill, int periodic) {
  const int np = periodic && !ctr[13] ? ctr[12] : 0;
  const long total = 6L * nf + np;
  for (long k = (long)blockIdx.x * GT + threadIdx.x; k < total; k += (long)gridDim.x * GT) {
    int u, v;
    if (k < 6L * nf) face_edge(faces, (int)(k / 6), (int)(k % 6), u, v);
    else u = prow[k - 6L * nf];
    atomicAdd(&deg[u], 1);
  }
  for (int i = blockIdx.x * GT + threadIdx.x; i < n; i += gridDim.x * GT) fill[i] = 0;
}

// Exclusive prefix sum of a[0..n) into a (a[n] = total), three passes (block sums, their scan
// in one block, add-back).  Integer, so the result is exact.
__global__ __launch_bounds__(256) void scan_local_kernel(int n, int* __restrict__ a, int* __restrict__ bsum) {
  __shared__ int s[SCAN_BLOCK];
  const int base = blockIdx.x * SCAN_BLOCK;
  for (int i = threadIdx.x; i < SCAN_BLOCK; i += 256) s[i] = base + i < n ? a[base + i] : 0;
  __syncthreads();
  // Hillis-Steele over 1024 entries, 4 per thread
  for (int off = 1; off < SCAN_BLOCK; off <<= 1) {
    int t[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = threadIdx.x + 256 * u;
      t[u] = i >= off ? s[i - off] : 0;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; ++u) s[threadIdx.x + 256 * u] += t[u];
    __syncthreads();
  }
  for (int i = threadIdx.x; i < SCAN_BLOCK; i += 256)
    if (base + i < n) a[base + i] = i ? s[i - 1] : 0;   // exclusive within the block
  if (threadIdx.x == 0) bsum[blockIdx.x] = s[SCAN_BLOCK - 1];
}

__global__ __launch_bounds__(1024) void scan_blocks_kernel(int nb, int* __restrict__ bsum) {
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int b = 0; b < nb; ++b) {
      const int v = bsum[b];
      bsum[b] = acc;
      acc += v;
    }
    bsum[nb] = acc;
  }
}

__global__ __launch_bounds__(256) void scan_add_kernel(int n, int* __restrict__ a, const int* __restrict__ bsum, int nb) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) a[i] += bsum[i / SCAN_BLOCK];
  if (i == 0) a[n] = bsum[nb];
}

__global__ __launch_bounds__(GT) void fill_kernel(int nf, const int64_t* __restrict__ faces, const int* __restrict__ ctr,
                                                  const int* __restrict__ prow, const int* __restrict__ pcol,
                                                  const int* __restrict__ off, int* __restrict__ fill,
                                                  int* __restrict__ nb, int periodic) {
  const int np = periodic && !ctr[13] ? ctr[12] : 0;
  const long total = 6L * nf + np;
  for (long k = (long)blockIdx.x * GT + threadIdx.x; k < total; k += (long)gridDim.x * GT) {
    int u, v, flag = 0;
    if (k < 6L * nf) {
      face_edge(faces, (int)(k / 6), (int)(k % 6), u, v);
    } else {
      u = prow[k - 6L * nf];
      v = pcol[k - 6L * nf];
      flag = 1;
    }
    nb[off[u] + atomicAdd(&fill[u], 1)] = 2 * v + flag;
  }
}

// Sort each row's slots (insertion sort: rows are short), count the distinct columns.
__global__ __launch_bounds__(GT) void row_sort_kernel(int n, const int* __restrict__ off, int* __restrict__ nb,
                                                      int* __restrict__ ucnt) {
  for (int r = blockIdx.x * GT + threadIdx.x; r < n; r += gridDim.x * GT) {
    int* a = nb + off[r];
    const int m = off[r + 1] - off[r];
    for (int i = 1; i < m; ++i) {
      const int x = a[i];
      int j = i - 1;
      while (j >= 0 && a[j] > x) {
        a[j + 1] = a[j];
        --j;
      }
      a[j + 1] = x;
    }
    int u = 0;
    for (int i = 0; i < m; ++i) u += i == 0 || (a[i] >> 1) != (a[i - 1] >> 1);
    ucnt[r] = u;
  }
}

// Emit row r's distinct columns at rowptr[r]: attribute = length if any slot of the column
// came from a face (flag 0; it sorts first), else 0.
__global__ __launch_bounds__(GT) void emit_kernel(int n, const float* __restrict__ p, int dim,
                                                  const int* __restrict__ off, const int* __restrict__ nb,
                                                  const int* __restrict__ rowptr, int64_t* __restrict__ rows,
                                                  int64_t* __restrict__ cols, float* __restrict__ attr) {
  for (int r = blockIdx.x * GT + threadIdx.x; r < n; r += gridDim.x * GT) {
    const int* a = nb + off[r];
    const int m = off[r + 1] - off[r];
    int k = rowptr[r];
    for (int i = 0; i < m; ++i) {
      const int v = a[i] >> 1;
      if (i > 0 && v == (a[i - 1] >> 1)) continue;
      float len = 0.f;
      if ((a[i] & 1) == 0) {   // a mesh edge: |pos[r] - pos[v]| (datasets.py:182-188)
        // torch.linalg.vector_norm's CPU order: s = t0 * t0, then s = fma(tk, tk, s), then sqrt
        float s = 0.f;
        for (int d = 0; d < dim; ++d) {
          const float t = p[(size_t)r * dim + d] - p[(size_t)v * dim + d];
          s = d == 0 ? nmul(t, t) : fmaf(t, t, s);
        }
        len = __fsqrt_rn(s);
      }
      rows[k] = r;
      cols[k] = v;
      attr[k] = len;
      ++k;
    }
  }
}

__global__ void finish_kernel(int n, const int* __restrict__ ctr, const int* __restrict__ rowptr, int periodic,
                              int* __restrict__ n_edges) {
  *n_edges = periodic && ctr[13] ? -1 : rowptr[n];
}

size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

size_t layout(int n, int nf, Scratch* s, char* base) {
  size_t o = 0;
  auto take = [&](size_t bytes) {
    char* p = base ? base + o : nullptr;
    o += align_up(bytes);
    return p;
  };
  const int nscan = (n + SCAN_BLOCK - 1) / SCAN_BLOCK + 1;
  const size_t pmax = 4 * (size_t)SIDE_MAX + 4;
  float* bbox = (float*)take(4 * sizeof(float) * BBOX_BLOCKS);
  int* ctr = (int*)take(16 * sizeof(int));
  int* side = (int*)take(4 * sizeof(int) * SIDE_MAX);
  int* prow = (int*)take(sizeof(int) * pmax);
  int* pcol = (int*)take(sizeof(int) * pmax);
  int* deg = (int*)take(sizeof(int) * ((size_t)n + 1));
  int* fill = (int*)take(sizeof(int) * (size_t)n);
  int* ucnt = (int*)take(sizeof(int) * ((size_t)n + 1));
  int* bsum = (int*)take(sizeof(int) * (size_t)(nscan + 1));
  int* nbp = (int*)take(sizeof(int) * (6 * (size_t)nf + pmax));
  if (s) *s = Scratch{bbox, ctr, side, prow, pcol, deg, fill, ucnt, bsum, nbp};
  return o;
}

int grid_for(long work) {
  long g = (work + GT - 1) / GT;
  const long cap = (long)device_cus() * 8;
  return (int)(g < 1 ? 1 : g > cap ? cap : g);
}

void scan(int n, int* a, int* bsum, hipStream_t st) {
  const int nb = (n + SCAN_BLOCK - 1) / SCAN_BLOCK;
  hipLaunchKernelGGL(scan_local_kernel, dim3(nb > 0 ? nb : 1), dim3(256), 0, st, n, a, bsum);
  hipLaunchKernelGGL(scan_blocks_kernel, dim3(1), dim3(1024), 0, st, nb, bsum);
  hipLaunchKernelGGL(scan_add_kernel, dim3((n + 256) / 256), dim3(256), 0, st, n, a, bsum, nb);
}

}  // namespace

extern "C" long pdg_mesh_graph_scratch_bytes(int n_nodes, int n_faces) {
  if (n_nodes <= 0 || n_faces < 0) return -1;
  return (long)layout(n_nodes, n_faces, nullptr, nullptr);
}

extern "C" int pdg_mesh_graph(int n_nodes, const float* points, int dim, int n_faces, const int64_t* faces,
                              int periodic, int64_t* edge_rows, int64_t* edge_cols, float* edge_attr, long capacity,
                              int* n_edges, void* scratch, long scratch_bytes, void* stream) {
  PDG_CHECK_ARG(n_nodes > 0 && n_faces >= 0 && (dim == 2 || dim == 3), "pdg_mesh_graph: bad sizes");
  PDG_CHECK_ARG(points && edge_rows && edge_cols && edge_attr && n_edges && scratch && (faces || n_faces == 0),
                "pdg_mesh_graph: null argument");
  PDG_CHECK_ARG(scratch_bytes >= pdg_mesh_graph_scratch_bytes(n_nodes, n_faces), "pdg_mesh_graph: scratch too small");
  PDG_CHECK_ARG(capacity >= 6L * n_faces + (periodic ? 4L * SIDE_MAX + 4 : 0),
                "pdg_mesh_graph: capacity below 6 * faces (+ periodic pairs)");
  PDG_CHECK_ARG((long)n_nodes * 2 + 1 < 0x7fffffffL && 6L * n_faces + 4L * SIDE_MAX + 4 < 0x7fffffffL,
                "pdg_mesh_graph: sizes beyond int32 indexing");
  hipStream_t st = (hipStream_t)stream;
  Scratch s;
  layout(n_nodes, n_faces, &s, (char*)scratch);
  const int nbb = (int)std::min<long>(BBOX_BLOCKS, (n_nodes + GT - 1) / GT);
  hipLaunchKernelGGL(bbox_kernel, dim3(nbb), dim3(GT), 0, st, n_nodes, points, dim, s.bbox, s.ctr);
  if (periodic) {
    hipLaunchKernelGGL(sides_kernel, dim3(grid_for(n_nodes)), dim3(GT), 0, st, n_nodes, points, dim, s.bbox, nbb,
                       s.ctr, s.side);
    hipLaunchKernelGGL(pairs_kernel, dim3(1), dim3(SORT_THREADS), 0, st, points, dim, s.ctr, s.side, s.prow, s.pcol);
  }
  (void)hipMemsetAsync(s.deg, 0, sizeof(int) * ((size_t)n_nodes + 1), st);
  const long work = 6L * n_faces + (periodic ? 4L * SIDE_MAX + 4 : 0);
  hipLaunchKernelGGL(count_kernel, dim3(grid_for(std::max<long>(work, n_nodes))), dim3(GT), 0, st, n_nodes, n_faces,
                     faces, s.ctr, s.prow, s.deg, s.fill, periodic);
  scan(n_nodes, s.deg, s.bsum, st);
  hipLaunchKernelGGL(fill_kernel, dim3(grid_for(work)), dim3(GT), 0, st, n_faces, faces, s.ctr, s.prow, s.pcol, s.deg,
                     s.fill, s.nb, periodic);
  hipLaunchKernelGGL(row_sort_kernel, dim3(grid_for(n_nodes)), dim3(GT), 0, st, n_nodes, s.deg, s.nb, s.ucnt);
  scan(n_nodes, s.ucnt, s.bsum, st);
  hipLaunchKernelGGL(emit_kernel, dim3(grid_for(n_nodes)), dim3(GT), 0, st, n_nodes, points, dim, s.deg, s.nb, s.ucnt,
                     edge_rows, edge_cols, edge_attr);
  hipLaunchKernelGGL(finish_kernel, dim3(1), dim3(1), 0, st, n_nodes, s.ctr, s.ucnt, periodic, n_edges);
  PDG_CHECK_LAUNCH("pdg_mesh_graph");
  return PDG_OK;
}
