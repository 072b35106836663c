// Device-side minibatch assembly: PyG collate of graphs that
// are resident in HBM (gnn_train.py:387-394 DataLoader -> Batch.from_data_list).
//
// Every batched array is a concatenation of per-graph segments, integer index
// arrays shifted by the graph's node / edge / nonzero offset in the batch.  The
// per-graph plan pieces (dst-sorted CSR, source grouping, divergence CSR and
// CSR^T) are precomputed once per graph with graph-local indices, so the batch
// plan needs no sort: graphs occupy disjoint, increasing node ranges, and the
// stable (dst, src) order of the batch is the concatenation of the graphs'
// own orders.  One launch copies all segments of all arrays from a job table.
#include "pdg_common.hpp"
#include "pdg_runtime.hpp"

using namespace pdg;

namespace {

__global__ __launch_bounds__(256) void collate_kernel(const pdg_copy_job* __restrict__ jobs, int njobs) {
  const int jb = blockIdx.y;
  if (jb >= njobs) return;
  const pdg_copy_job jbd = jobs[jb];
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < jbd.count; i += stride) {
    switch (jbd.kind) {
      case PDG_COPY_B32:
        reinterpret_cast<int*>(jbd.dst)[i] = reinterpret_cast<const int*>(jbd.src)[i] + (int)jbd.add;
        break;
      case PDG_COPY_B64:
        reinterpret_cast<long long*>(jbd.dst)[i] = reinterpret_cast<const long long*>(jbd.src)[i] + jbd.add;
        break;
      default:   // PDG_COPY_F32 (bit copy; add ignored)
        reinterpret_cast<unsigned*>(jbd.dst)[i] = reinterpret_cast<const unsigned*>(jbd.src)[i];
        break;
    }
  }
}

}  // namespace

extern "C" int pdg_collate(const pdg_copy_job* jobs, int njobs, long max_count, void* stream) {
  PDG_CHECK_ARG(njobs >= 0 && njobs <= 65535, "pdg_collate: njobs must be in [0, 65535]");
  if (njobs == 0 || max_count <= 0) return PDG_OK;
  long bx = (max_count + 255) / 256;
  if (bx > 256) bx = 256;
  hipLaunchKernelGGL(collate_kernel, dim3((unsigned)bx, (unsigned)njobs), dim3(256), 0, (hipStream_t)stream, jobs,
                     njobs);
  PDG_CHECK_LAUNCH("pdg_collate");
  return PDG_OK;
}
