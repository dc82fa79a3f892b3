// fq_vit MinmaxObserver.update on the GPU: running per-row / per-column /
// whole-tensor max and min of a calibration tensor.
//
// Reference: fq_vit/models/ptq/observer/minmax.py:14-29 (update: cur_max / cur_min over dim 1 of
// the reshaped tensor, merged with the running values, reduced to a scalar for layer_wise) and
// observer/base.py:16-29 (reshape_tensor: weights (out, -1) -> stats per row; activations
// channel-last (-1, C).T -> stats per column).  HBM-bound reductions; max/min are exact in any
// order, so results are bit-identical to torch's.  NaN propagates like torch.max / torch.min.
#include "common.h"

namespace samq {

__device__ __forceinline__ float nan_max(float a, float b) { return (a != a || a > b) ? a : b; }
__device__ __forceinline__ float nan_min(float a, float b) { return (a != a || a < b) ? a : b; }

template <bool F16>
__device__ __forceinline__ float mm_load(const void* x, int64_t i) {
  if (F16) return (float)((const _Float16*)x)[i];
  return ((const float*)x)[i];
}

// stats per row: one wave per row, lanes stride the row
template <bool F16>
__global__ __launch_bounds__(256) void mm_rows_kernel(const void* __restrict__ x, int64_t rows, int C,
                                                      float* __restrict__ max_io, float* __restrict__ min_io,
                                                      int init) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float mx = -INFINITY, mn = INFINITY;
  bool nan = false;
  for (int c = lane; c < C; c += 64) {
    const float v = mm_load<F16>(x, row * C + c);
    nan |= v != v;
    mx = fmaxf(mx, v);
    mn = fminf(mn, v);
  }
  mx = wave_max(mx);
  mn = -wave_max(-mn);
  if (__any(nan)) mx = mn = __builtin_nanf("");
  if (lane == 0) {
    max_io[row] = init ? mx : nan_max(mx, max_io[row]);
    min_io[row] = init ? mn : nan_min(mn, min_io[row]);
  }
}

// stats per column, pass 1: thread = column, blockIdx.y = slab of rows -> ws[split][C]
template <bool F16>
__global__ __launch_bounds__(256) void mm_cols_kernel(const void* __restrict__ x, int64_t rows, int C,
                                                      int64_t rows_per_split, float* __restrict__ ws_max,
                                                      float* __restrict__ ws_min) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_split;
  const int64_t r1 = r0 + rows_per_split < rows ? r0 + rows_per_split : rows;
  float mx = -INFINITY, mn = INFINITY;
  bool nan = false;
  for (int64_t r = r0; r < r1; ++r) {
    const float v = mm_load<F16>(x, r * C + c);
    nan |= v != v;
    mx = fmaxf(mx, v);
    mn = fminf(mn, v);
  }
  if (nan) mx = mn = __builtin_nanf("");
  ws_max[(int64_t)blockIdx.y * C + c] = mx;
  ws_min[(int64_t)blockIdx.y * C + c] = mn;
}

// pass 2, per column: fold the splits and the running values
__global__ __launch_bounds__(256) void mm_merge_cols_kernel(const float* __restrict__ ws_max,
                                                            const float* __restrict__ ws_min, int splits, int C,
                                                            float* __restrict__ max_io, float* __restrict__ min_io,
                                                            int init) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  float mx = ws_max[c], mn = ws_min[c];
  for (int s = 1; s < splits; ++s) {
    mx = nan_max(mx, ws_max[(int64_t)s * C + c]);
    mn = nan_min(mn, ws_min[(int64_t)s * C + c]);
  }
  max_io[c] = init ? mx : nan_max(mx, max_io[c]);
  min_io[c] = init ? mn : nan_min(mn, min_io[c]);
}

// pass 2, whole tensor: one workgroup folds every partial into the running scalar
__global__ __launch_bounds__(256) void mm_merge_all_kernel(const float* __restrict__ ws_max,
                                                           const float* __restrict__ ws_min, int64_t n,
                                                           float* __restrict__ max_io, float* __restrict__ min_io,
                                                           int init) {
  __shared__ float smx[4], smn[4];
  __shared__ int snan[4];
  float mx = -INFINITY, mn = INFINITY;
  bool nan = false;
  for (int64_t i = threadIdx.x; i < n; i += 256) {
    const float a = ws_max[i], b = ws_min[i];
    nan |= (a != a) | (b != b);
    mx = fmaxf(mx, a);
    mn = fminf(mn, b);
  }
  mx = wave_max(mx);
  mn = -wave_max(-mn);
  const int wnan = __any(nan) ? 1 : 0;
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { smx[w] = mx; smn[w] = mn; snan[w] = wnan; }
  __syncthreads();
  if (threadIdx.x == 0) {
    mx = smx[0];
    mn = smn[0];
    for (int i = 1; i < 4; ++i) { mx = fmaxf(mx, smx[i]); mn = fminf(mn, smn[i]); }
    if (snan[0] | snan[1] | snan[2] | snan[3]) mx = mn = __builtin_nanf("");
    max_io[0] = init ? mx : nan_max(mx, max_io[0]);
    min_io[0] = init ? mn : nan_min(mn, min_io[0]);
  }
}

static int64_t mm_splits(int64_t rows, int C) {
  // enough row slabs to put ~2 K workgroups on the chip, at least 64 rows each
  const int64_t col_blocks = (C + 255) / 256;
  int64_t s = (2048 + col_blocks - 1) / col_blocks;
  const int64_t max_s = (rows + 63) / 64;
  s = s < max_s ? s : max_s;
  return s < 1 ? 1 : (s > 1024 ? 1024 : s);
}

}  // namespace samq

using namespace samq;

extern "C" size_t samq_minmax_workspace(int64_t rows, int C, int axis) {
  if (axis == SAMQ_MM_PER_ROW || rows <= 0 || C <= 0) return 0;
  return (size_t)(2 * mm_splits(rows, C) * C);
}

extern "C" int samq_minmax(const void* x, int64_t rows, int C, int in_f16, int axis, float* max_io, float* min_io,
                           int init, float* workspace, size_t workspace_floats, hipStream_t stream) {
  SAMQ_REQUIRE(x && max_io && min_io, SAMQ_ERR_INVALID, "minmax: null pointer");
  SAMQ_REQUIRE(rows > 0 && C > 0, SAMQ_ERR_INVALID, "minmax: empty tensor (torch.max would raise)");
  SAMQ_REQUIRE(axis == SAMQ_MM_PER_ROW || axis == SAMQ_MM_PER_COL || axis == SAMQ_MM_ALL, SAMQ_ERR_INVALID,
               "minmax: axis must be SAMQ_MM_PER_ROW, SAMQ_MM_PER_COL or SAMQ_MM_ALL");
  if (axis == SAMQ_MM_PER_ROW) {
    const dim3 grid((unsigned)((rows + 3) / 4));
    if (in_f16) hipLaunchKernelGGL((mm_rows_kernel<true>), grid, dim3(256), 0, stream, x, rows, C, max_io, min_io, init);
    else hipLaunchKernelGGL((mm_rows_kernel<false>), grid, dim3(256), 0, stream, x, rows, C, max_io, min_io, init);
    SAMQ_LAUNCH_CHECK("minmax rows launch");
    return SAMQ_OK;
  }
  const int64_t splits = mm_splits(rows, C);
  SAMQ_REQUIRE(workspace && workspace_floats >= (size_t)(2 * splits * C), SAMQ_ERR_INVALID,
               "minmax: workspace smaller than samq_minmax_workspace()");
  const int64_t rps = (rows + splits - 1) / splits;
  float* ws_max = workspace;
  float* ws_min = workspace + splits * C;
  const dim3 grid((unsigned)((C + 255) / 256), (unsigned)splits);
  if (in_f16) hipLaunchKernelGGL((mm_cols_kernel<true>), grid, dim3(256), 0, stream, x, rows, C, rps, ws_max, ws_min);
  else hipLaunchKernelGGL((mm_cols_kernel<false>), grid, dim3(256), 0, stream, x, rows, C, rps, ws_max, ws_min);
  SAMQ_LAUNCH_CHECK("minmax cols launch");
  if (axis == SAMQ_MM_PER_COL)
    hipLaunchKernelGGL(mm_merge_cols_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, stream, ws_max, ws_min,
                       (int)splits, C, max_io, min_io, init);
  else
    hipLaunchKernelGGL(mm_merge_all_kernel, dim3(1), dim3(256), 0, stream, ws_max, ws_min, splits * C, max_io, min_io,
                       init);
  SAMQ_LAUNCH_CHECK("minmax merge launch");
  return SAMQ_OK;
}
