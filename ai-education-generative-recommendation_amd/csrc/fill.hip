// Device fill used instead of hipMemsetAsync / hipMemsetD32Async.  The library's calls are meant to
// be captured into graphs (ops.SasTrainGraph, ops.SasTrainStepGraph); on this ROCm a captured
// memset node did not clear its buffer on the second and later replays (the dM buffer of the
// sampled BCE backward kept the previous step's gradient plus whatever reused its memory,
// profiles/r02_train_graph_diag.txt), while kernel nodes replay exactly.
#include "gr_common.h"

namespace gr {

__global__ __launch_bounds__(256) void fill32_kernel(uint32_t* __restrict__ p, uint32_t v, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = v;
}

__global__ __launch_bounds__(256) void fill64_kernel(uint64_t* __restrict__ p, uint64_t v, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = v;
}

}  // namespace gr

int gr_fill32_launch(void* p, uint32_t value, int64_t count, hipStream_t st) {
  if (count <= 0) return GR_OK;
  int64_t blocks = (count + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(gr::fill32_kernel, dim3((unsigned)blocks), dim3(256), 0, st, reinterpret_cast<uint32_t*>(p),
                     value, count);
  return gr::check_launch("gr fill");
}

int gr_fill64_launch(void* p, uint64_t value, int64_t count, hipStream_t st) {
  if (count <= 0) return GR_OK;
  int64_t blocks = (count + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(gr::fill64_kernel, dim3((unsigned)blocks), dim3(256), 0, st, reinterpret_cast<uint64_t*>(p),
                     value, count);
  return gr::check_launch("gr fill64");
}
