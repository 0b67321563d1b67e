// treeinfer_kernels.h — gfx950 tree-traversal kernels (device code).
//
// Two layouts, one row per lane, one 64-wide wavefront walking the SAME tree
// at a time so tree data is shared across lanes:
//
//  * heap  : every tree padded to a complete binary tree of depth D (<= 8).
//            Children are implicit (2i+1 / 2i+2); a tree is one contiguous
//            record {internal nodes[2^D-1], leaves[2^D * leaf_width]} and the
//            workgroup stages S whole records at a time into LDS.  Each lane
//            walks 4 trees at once (4 independent LDS-latency chains) and adds
//            the leaves in tree order, so float32 sums are bit-identical to the
//            library's sequential loop.
//  * expl  : irregular / deep trees (LightGBM leaf-wise, sklearn depth 16).
//            Explicit child indices, nodes read from global memory (L2 / MALL
//            resident), a divergent while-loop per tree.
//
// Row features are staged once per 256-row tile into LDS as [feature][row]:
// lane l reads column f at LDS word f*R + l, so the 64 lanes of a ds_read_b32
// hit 64 distinct banks whatever feature each lane's node tests.
//
// The margin epilogue (base, average, sigmoid / softmax / argmax ...) is fused
// into the same launch: one kernel per predict.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "treeinfer.h"

namespace ti {

constexpr uint32_t kMetaNanLeft = 0x80000000u;
constexpr uint32_t kMetaZeroFlip = 0x40000000u;
constexpr uint32_t kMetaFeatMask = 0x00FFFFFFu;
constexpr int kMaxGroups = 16;

template <typename XT> struct HeapNode;
template <> struct HeapNode<float> { float thr; uint32_t meta; };                   // 8 B
template <> struct HeapNode<double> { double thr; uint32_t meta; uint32_t pad; };   // 16 B

struct ExpNode { float thr; uint32_t meta; int32_t left; int32_t right; };          // 16 B

// Kernel arguments (passed by value in the kernarg segment).
struct KArgs {
  const void* X;
  int64_t n_rows;
  int64_t row_stride;
  int32_t n_cols;
  int32_t n_features;
  int32_t n_trees;
  int32_t n_groups;
  int32_t leaf_width;
  int32_t kind;
  int32_t transform;
  int32_t base_first;
  int32_t lgb_zero_map;
  int32_t zero_rule;
  int32_t divide;
  int32_t depth;          // heap depth D
  int32_t stage_trees;    // heap: trees per LDS stage
  int32_t pad0;
  double transform_param;
  double average_divisor;
  double base[kMaxGroups];
  // heap layout
  const unsigned char* trees;     // [T][tree_stride]
  int64_t tree_stride;
  const int32_t* heap_leaf_ids;   // [T][2^D]
  // explicit layout
  const ExpNode* nodes;           // [n_internal]
  const double* thr64;            // [n_internal]
  const int64_t* node_base;       // [T]
  const int32_t* root;            // [T] >= 0 internal index, < 0 : ~leaf
  const int64_t* leaf_base;       // [T]
  const void* leaves;             // [n_leaves * leaf_width] ACC
  const int32_t* exp_leaf_ids;    // [n_leaves]
  // shared
  const int32_t* tree_group;      // [T]
  void* out;
};

__device__ __forceinline__ size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

__device__ __forceinline__ float t_exp(float x) { return expf(x); }
__device__ __forceinline__ double t_exp(double x) { return exp(x); }
__device__ __forceinline__ float t_log1p(float x) { return log1pf(x); }
__device__ __forceinline__ double t_log1p(double x) { return log1p(x); }

template <typename XT>
__device__ __forceinline__ XT nan_value();
template <> __device__ __forceinline__ float nan_value<float>() { return __builtin_nanf(""); }
template <> __device__ __forceinline__ double nan_value<double>() { return __builtin_nan(""); }

// LightGBM's predictor keeps only |x| > kZeroThreshold (1e-35f) or NaN
// entries of a dense row; everything else reads as 0.0.
template <typename XT>
__device__ __forceinline__ XT zero_map(XT v, int on) {
  return (on && __builtin_fabs((double)v) <= (double)1e-35f) ? XT(0) : v;
}

// Canonical split rule (treeinfer.h): left iff x <= thr, NaN by flag,
// x == 0 flipped for LightGBM Zero-missing nodes whose default differs.
template <typename XT, typename TT>
__device__ __forceinline__ bool go_left(XT x, TT thr, uint32_t meta, int zero_rule) {
  bool left = x <= thr;
  const bool nanx = x != x;
  left = nanx ? ((meta & kMetaNanLeft) != 0) : left;
  if (zero_rule) {
    const bool flip = (x == XT(0)) && ((meta & kMetaZeroFlip) != 0);
    left = flip ? !left : left;
  }
  return left;
}

// Stage the tile's features into LDS as [f][R].  Columns >= n_cols read NaN
// (missing), matching a DMatrix narrower than the booster.
template <typename XT>
__device__ __forceinline__ void stage_features(XT* feat, const KArgs& a, int64_t row0, int R, int tid) {
  const XT* X = static_cast<const XT*>(a.X);
  const int F = a.n_features;
  const int C = a.n_cols;
  const int FC = F < C ? F : C;
  const int64_t left_rows = a.n_rows - row0;
  const int rows_here = left_rows < R ? (int)left_rows : R;
  if (a.row_stride == C) {
    // the tile is one contiguous span: consecutive lanes read consecutive words
    const XT* base = X + row0 * (int64_t)C;
    const uint32_t n = (uint32_t)rows_here * (uint32_t)C;
    const uint32_t uC = (uint32_t)C;
    for (uint32_t e = tid; e < n; e += R) {
      const uint32_t r = e / uC;
      const uint32_t c = e - r * uC;
      if ((int)c < F) feat[c * R + r] = zero_map(base[e], a.lgb_zero_map);
    }
  } else if (tid < rows_here) {
    const XT* xr = X + (row0 + tid) * a.row_stride;
    for (int c = 0; c < FC; ++c) feat[c * R + tid] = zero_map(xr[c], a.lgb_zero_map);
  }
  for (int c = FC; c < F; ++c) feat[c * R + tid] = nan_value<XT>();
}

// Feature fetch for a lane: LDS image, or straight from the row (very wide F).
template <typename XT, bool FEAT_LDS>
__device__ __forceinline__ XT fetch(const XT* feat, const XT* xrow, uint32_t f, int R, int tid,
                                    const KArgs& a) {
  if (FEAT_LDS) {
    return feat[f * R + tid];
  } else {
    return (int)f < a.n_cols ? zero_map(xrow[f], a.lgb_zero_map) : nan_value<XT>();
  }
}

template <typename ACC, int KMAX>
__device__ __forceinline__ void add_leaf(ACC (&acc)[KMAX], const ACC* lv, int leaf, int LW, int g) {
  if (KMAX == 1) {
    acc[0] += lv[leaf];
  } else if (LW == 1) {
    const ACC v = lv[leaf];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) acc[k] = (k == g) ? acc[k] + v : acc[k];
  } else {
    const ACC* p = lv + (int64_t)leaf * LW;
#pragma unroll
    for (int k = 0; k < KMAX; ++k)
      if (k < LW) acc[k] += p[k];
  }
}

template <typename ACC, int KMAX>
__device__ __forceinline__ void init_acc(ACC (&acc)[KMAX], const KArgs& a) {
#pragma unroll
  for (int k = 0; k < KMAX; ++k) acc[k] = a.base_first ? (ACC)a.base[k] : ACC(0);
}

// Margin epilogue + output transform for one row, in the accumulator's
// precision (float32 for XGBoost, float64 for LightGBM / sklearn).
template <typename ACC, int KMAX>
__device__ __forceinline__ void finish_row(const ACC (&acc)[KMAX], const KArgs& a, int64_t row) {
  const int K = a.n_groups;
  ACC m[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    ACC v = acc[k];
    if (!a.base_first) v = (ACC)a.base[k] + v;   // xgboost 0.82: preds(base) += psum
    if (a.divide) v = v / (ACC)a.average_divisor;
    m[k] = v;
  }
  ACC* out = static_cast<ACC*>(a.out);
  const int tr = a.kind == TI_OUTPUT_MARGIN ? TI_TRANSFORM_IDENTITY : a.transform;
  if (tr == TI_TRANSFORM_ARGMAX) {
    int best = 0;
#pragma unroll
    for (int k = 1; k < KMAX; ++k)
      if (k < K && m[best] < m[k]) best = k;     // first maximum (std::max_element)
    out[row] = (ACC)best;
    return;
  }
  ACC* o = out + row * K;
  if (tr == TI_TRANSFORM_SOFTMAX) {
    ACC wmax = m[0];
#pragma unroll
    for (int k = 1; k < KMAX; ++k)
      if (k < K) wmax = (m[k] < wmax) ? wmax : m[k];   // std::max(rec[i], wmax)
    double wsum = 0.0;
#pragma unroll
    for (int k = 0; k < KMAX; ++k)
      if (k < K) {
        m[k] = t_exp(m[k] - wmax);
        wsum += m[k];
      }
#pragma unroll
    for (int k = 0; k < KMAX; ++k)
      if (k < K) o[k] = m[k] / (ACC)wsum;
    return;
  }
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    if (k >= K) continue;
    ACC v = m[k];
    switch (tr) {
      case TI_TRANSFORM_SIGMOID:
        v = ACC(1) / (ACC(1) + t_exp(-((ACC)a.transform_param * v)));
        break;
      case TI_TRANSFORM_HINGE:
        v = v > ACC(0) ? ACC(1) : ACC(0);
        break;
      case TI_TRANSFORM_EXP:
        v = t_exp(v);
        break;
      case TI_TRANSFORM_SIGNSQUARE:
        v = (ACC)((v > ACC(0)) - (v < ACC(0))) * v * v;
        break;
      case TI_TRANSFORM_LOG1PEXP:
        v = t_log1p(t_exp(v));
        break;
      default:
        break;
    }
    o[k] = v;
  }
}

// ---------------------------------------------------------------- heap kernel
template <typename XT, typename ACC, int KMAX, bool FEAT_LDS>
__global__ void __launch_bounds__(256) heap_predict_kernel(const KArgs a) {
  using Node = HeapNode<XT>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int R = blockDim.x;
  const int tid = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * R;
  const int64_t row = row0 + tid;
  const bool live = row < a.n_rows;
  XT* feat = reinterpret_cast<XT*>(smem);
  const size_t feat_bytes = FEAT_LDS ? align16((size_t)a.n_features * R * sizeof(XT)) : 0;
  unsigned char* stage = smem + feat_bytes;
  const XT* xrow = static_cast<const XT*>(a.X) + (live ? row : a.n_rows - 1) * a.row_stride;
  if (FEAT_LDS) stage_features<XT>(feat, a, row0, R, tid);

  const int D = a.depth;
  const int NI = (1 << D) - 1;
  const int NL = 1 << D;
  const int T = a.n_trees;
  const int S = a.stage_trees;
  const int64_t stride = a.tree_stride;
  const bool want_leaf = a.kind == TI_OUTPUT_LEAF;
  int32_t* out_leaf = static_cast<int32_t*>(a.out);

  ACC acc[KMAX];
  init_acc(acc, a);

  for (int t0 = 0; t0 < T; t0 += S) {
    const int cnt = (T - t0) < S ? (T - t0) : S;
    __syncthreads();   // previous stage fully consumed (and features staged)
    {
      const uint4* src = reinterpret_cast<const uint4*>(a.trees + (int64_t)t0 * stride);
      uint4* dst = reinterpret_cast<uint4*>(stage);
      const int n16 = (int)(((int64_t)cnt * stride) >> 4);
      for (int i = tid; i < n16; i += R) dst[i] = src[i];
    }
    __syncthreads();
    for (int j = 0; j < cnt; j += 4) {
      const unsigned char* tp[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) tp[q] = stage + (int64_t)((j + q) < cnt ? (j + q) : (cnt - 1)) * stride;
      uint32_t idx[4] = {0u, 0u, 0u, 0u};
      for (int l = 0; l < D; ++l) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const Node nd = reinterpret_cast<const Node*>(tp[q])[idx[q]];
          const XT x = fetch<XT, FEAT_LDS>(feat, xrow, nd.meta & kMetaFeatMask, R, tid, a);
          const bool left = go_left(x, (XT)nd.thr, nd.meta, a.zero_rule);
          idx[q] = 2u * idx[q] + (left ? 1u : 2u);
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (j + q < cnt) {
          const int leaf = (int)idx[q] - NI;
          const int t = t0 + j + q;
          if (want_leaf) {
            if (live) out_leaf[row * T + t] = a.heap_leaf_ids[(int64_t)t * NL + leaf];
          } else {
            const ACC* lv = reinterpret_cast<const ACC*>(tp[q] + (size_t)NI * sizeof(Node));
            add_leaf<ACC, KMAX>(acc, lv, leaf, a.leaf_width, a.tree_group[t]);
          }
        }
      }
    }
  }
  if (!live || want_leaf) return;
  finish_row<ACC, KMAX>(acc, a, row);
}

// ------------------------------------------------------------ explicit kernel
template <typename XT, typename ACC, int KMAX, bool FEAT_LDS>
__global__ void __launch_bounds__(256) explicit_predict_kernel(const KArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int R = blockDim.x;
  const int tid = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * R;
  const int64_t row = row0 + tid;
  const bool live = row < a.n_rows;
  XT* feat = reinterpret_cast<XT*>(smem);
  const XT* xrow = static_cast<const XT*>(a.X) + (live ? row : a.n_rows - 1) * a.row_stride;
  if (FEAT_LDS) {
    stage_features<XT>(feat, a, row0, R, tid);
    __syncthreads();
  }
  const int T = a.n_trees;
  const bool want_leaf = a.kind == TI_OUTPUT_LEAF;
  int32_t* out_leaf = static_cast<int32_t*>(a.out);
  const ACC* leaves = static_cast<const ACC*>(a.leaves);

  ACC acc[KMAX];
  init_acc(acc, a);

  for (int t = 0; t < T; ++t) {
    const int64_t nb = a.node_base[t];
    const ExpNode* nodes = a.nodes + nb;
    int32_t c = a.root[t];
    while (c >= 0) {
      const ExpNode nd = nodes[c];
      const XT x = fetch<XT, FEAT_LDS>(feat, xrow, nd.meta & kMetaFeatMask, R, tid, a);
      bool left;
      if (sizeof(XT) == 4) {
        left = go_left(x, (XT)nd.thr, nd.meta, a.zero_rule);
      } else {
        left = go_left(x, (XT)a.thr64[nb + c], nd.meta, a.zero_rule);
      }
      c = left ? nd.left : nd.right;
    }
    const int64_t lb = a.leaf_base[t];
    if (want_leaf) {
      if (live) out_leaf[row * T + t] = a.exp_leaf_ids[lb + (~c)];
    } else {
      add_leaf<ACC, KMAX>(acc, leaves + lb * a.leaf_width, ~c, a.leaf_width, a.tree_group[t]);
    }
  }
  if (!live || want_leaf) return;
  finish_row<ACC, KMAX>(acc, a, row);
}

}  // namespace ti
