// treeinfer_kernels.h — gfx950 tree-traversal kernels (device code).
//
// One row per lane; all 64 lanes of a wavefront walk the SAME tree at a time,
// so tree data is shared by the whole workgroup.  Two layouts:
//
//  * heap  : every tree padded to a complete binary tree of depth D (<= 8).
//            Children are implicit (2i+1 / 2i+2); a tree is one contiguous
//            record {internal nodes[2^D-1], leaves[2^D * leaf_width]}.  The
//            workgroup copies S whole records at a time into LDS; each lane
//            then walks TILP trees at once (TILP independent LDS-latency
//            chains) and adds their leaves in tree order, so float32 sums are
//            bit-identical to the library's sequential loop.
//  * expl  : irregular / deep trees (LightGBM leaf-wise, sklearn depth 16).
//            Explicit child indices, nodes read from global memory (L2 / MALL
//            resident), a divergent while-loop per tree.
//
// Row features are staged once per tile into LDS as [feature][row]: lane l
// reads column f at byte f*R*sizeof(XT) + l*sizeof(XT), so the lanes of a
// ds_read_b32 hit distinct banks whatever feature each lane's node tests.  In
// the heap layout a node's meta word carries that column byte offset directly
// (low 24 bits), so the feature address is one v_and_or of meta and the lane
// offset.
//
// The margin epilogue (base, average, sigmoid / softmax / argmax ...) is fused
// into the same launch: one kernel per predict.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "treeinfer.h"

#ifndef TI_TILP
#define TI_TILP 8   // trees walked concurrently per lane (heap layout)
#endif
#ifndef TI_ASM_STEP
#define TI_ASM_STEP 1   // binned heap: hand-scheduled compare/select/carry step
#endif
#ifndef TI_EXP_ILP
#define TI_EXP_ILP 4    // trees walked concurrently per lane (explicit kernels)
#endif
#ifndef TI_BTILP
#define TI_BTILP 4      // trees walked concurrently per lane (binned heap)
#endif
#ifndef TI_PF
#define TI_PF 8     // 16-byte words per thread prefetched for the next tree stage
#endif
#ifndef TI_BIN_Q
#define TI_BIN_Q 8   // binned heap: features binary-searched at once per lane (the temp
                     // area holds 8 columns of a 512-row tile: more would cost LDS)
#endif

namespace ti {

constexpr uint32_t kMetaNanLeft = 0x80000000u;
constexpr uint32_t kMetaZeroFlip = 0x40000000u;
constexpr uint32_t kMetaCat = 0x20000000u;        // explicit layout: categorical node
constexpr uint32_t kMetaFeatMask = 0x00FFFFFFu;
constexpr int kMaxGroups = 16;
constexpr int kExpIlp = TI_EXP_ILP;       // trees per lane in the global explicit kernels
constexpr int kTilp = TI_TILP;
constexpr int kBTilp = TI_BTILP;
constexpr int kPf = TI_PF;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));   // native vector: stays in VGPRs

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
  int32_t divide;
  int32_t depth;          // heap depth D
  int32_t stage_trees;    // heap: trees per LDS stage
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
  const uint32_t* cat_words;      // categorical bitsets: [nwords, w0, w1, ...] per node
  // staged record layouts (7, 9)
  const int32_t* stage_start;     // [n_stages+1] first tree of each LDS stage
  int32_t n_stages;
  // layout 9's compact u8 bottom (t8explicit_predict_kernel)
  const uint32_t* tx_pos;         // [T+1] first bottom position of each tree
  const void* tx_vals;            // [positions] leaf value (ACC)
  const int32_t* tx_ord;          // [positions] leaf ordinal in its tree
  // binned layouts: rank images of the features (see stage_bins)
  const void* bin_tbl;            // [F][2^bin_L] Eytzinger threshold tables, XT
  int32_t bin_L;                  // search depth (common to all features)
  int32_t bin_kary;               // > 0: float32 5-ary search tables of this height (rx_stage_bins)
  int32_t bin_words;              // packed bin words per row (C)
  int32_t bin_chunk;              // columns binned per pass through the temp area
  int32_t stage_off;              // LDS byte offset of the tree stage / temp area
  uint32_t bin_mask;              // binned heap: the node word's bin-offset bits
  // record explicit layout (6): 8-byte slots, first slot of each tree
  const uint2* rx_recs;           // [slots]
  const uint32_t* rx_base;        // [T] first slot of each tree
  const uint32_t* rx_nint;        // [T] internal slots of each tree (leaves follow)
  uint32_t rx_slots;              // slots in rx_recs
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

// Canonical split rule (treeinfer.h): left iff x <= thr; a NaN goes left iff
// the node's NaN bit (meta bit 31) is set; with ZERO, x == 0 flips the compare
// for LightGBM Zero-missing nodes whose default differs (meta bit 30).
// CHECK_NAN = false is the uniform fast path for tiles known to hold no NaN.
template <bool ZERO, bool CHECK_NAN = true, typename XT>
__device__ __forceinline__ bool go_left(XT x, XT thr, uint32_t meta) {
  bool left = x <= thr;
  if (CHECK_NAN) left = left || ((x != x) && (int32_t)meta < 0);
  if (ZERO) left = left != ((x == XT(0)) && (meta & kMetaZeroFlip) != 0);
  return left;
}

// LightGBM Tree::CategoricalDecision: v = (int)x; NaN, x <= -1 and
// x >= 2^31 (INT_MIN on the reference's x86) go right; otherwise left iff bit
// v is inside the node's bitset and set.  `bs` points at [nwords, w0, w1 ...].
__device__ __forceinline__ bool cat_left(const uint32_t* bs, double x) {
  if (!(x > -1.0 && x < 2147483648.0)) return false;
  const uint32_t v = static_cast<uint32_t>(x);
  const uint32_t w = v >> 5;
  if (w >= bs[0]) return false;
  return (bs[1 + w] >> (v & 31u)) & 1u;
}

// One heap node from LDS in a single wide read (ds_read_b64 / ds_read_b128).
__device__ __forceinline__ void load_node(const HeapNode<float>* p, float& thr, uint32_t& meta) {
  const uint2 v = *reinterpret_cast<const uint2*>(p);
  thr = __uint_as_float(v.x);
  meta = v.y;
}
__device__ __forceinline__ void load_node(const HeapNode<double>* p, double& thr, uint32_t& meta) {
  const uint4 v = *reinterpret_cast<const uint4*>(p);
  thr = __hiloint2double((int)v.y, (int)v.x);
  meta = v.z;
}

// The dynamic LDS region starts at LDS address 0 (no static __shared__ in
// these kernels), so a feature-image byte offset is already an LDS address.
template <typename XT>
__device__ __forceinline__ XT lds_at(uint32_t byte_addr) {
  return *reinterpret_cast<const __attribute__((address_space(3))) XT*>(
      static_cast<uintptr_t>(byte_addr));
}

// Stage the tile's features into LDS as [f][R].  Columns >= n_cols read NaN
// (missing), matching a DMatrix narrower than the booster.  Returns (uniformly
// across the workgroup) whether the tile holds a NaN; `flag` is a word of the
// dynamic LDS region (no static __shared__: see lds_at).  Ends in a barrier.
template <typename XT>
__device__ __forceinline__ bool stage_features(XT* feat, volatile int* flag, const KArgs& a,
                                               int64_t row0, int R, int tid) {
  if (tid == 0) *flag = 0;
  __syncthreads();
  const XT* X = static_cast<const XT*>(a.X);
  const int F = a.n_features;
  const int C = a.n_cols;
  const int FC = F < C ? F : C;
  const int64_t left_rows = a.n_rows - row0;
  const int rows_here = left_rows < R ? (int)left_rows : R;
  bool has_nan = false;
  if (a.row_stride == C) {
    // the tile is one contiguous span: consecutive lanes read consecutive words
    const XT* base = X + row0 * (int64_t)C;
    const uint32_t n = (uint32_t)rows_here * (uint32_t)C;
    const uint32_t uC = (uint32_t)C;
    for (uint32_t e = tid; e < n; e += R) {
      const uint32_t r = e / uC;
      const uint32_t c = e - r * uC;
      const XT v = base[e];
      if ((int)c < F) {
        feat[c * R + r] = zero_map(v, a.lgb_zero_map);
        has_nan |= v != v;
      }
    }
  } else if (tid < rows_here) {
    const XT* xr = X + (row0 + tid) * a.row_stride;
    for (int c = 0; c < FC; ++c) {
      const XT v = xr[c];
      feat[c * R + tid] = zero_map(v, a.lgb_zero_map);
      has_nan |= v != v;
    }
  }
  for (int c = FC; c < F; ++c) feat[c * R + tid] = nan_value<XT>();
  // rows past n_rows stay unwritten: their lanes compute and discard
  if (has_nan || FC < F) *flag = 1;
  __syncthreads();
  return *flag != 0;
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
      case TI_TRANSFORM_STEP:
        v = v >= ACC(0) ? ACC(1) : ACC(0);
        break;
      default:
        break;
    }
    o[k] = v;
  }
}

// Tree stages move global -> registers -> LDS.  The next stage's loads are
// issued before the current stage is walked and land in registers while the
// lanes traverse, so only the LDS write sits between two stages.  A stage is
// at most kPf * 16 * R bytes (the host sizes it so).
__device__ __forceinline__ void prefetch_stage(u32x4 (&pf)[kPf], const u32x4* __restrict__ src,
                                               int n16, int tid, int R) {
  // unconditional loads (index clamped inside the stage): no exec-masked
  // branches, so every load is in flight at once and pf stays in registers
#pragma unroll
  for (int u = 0; u < kPf; ++u) {
    const int i = tid + u * R;
    pf[u] = src[i < n16 ? i : n16 - 1];
  }
}
__device__ __forceinline__ void commit_stage(const u32x4 (&pf)[kPf], u32x4* __restrict__ dst,
                                             int n16, int tid, int R) {
#pragma unroll
  for (int u = 0; u < kPf; ++u) {
    const int i = tid + u * R;
    if (i < n16) dst[i] = pf[u];
  }
}

// ---------------------------------------------------------------- heap kernel
// meta bits 0..23 hold the node's feature as a byte offset: into the LDS
// feature image (FEAT_LDS) or into the row (global fallback for very wide F).
template <typename XT, typename ACC, int KMAX, bool FEAT_LDS, bool ZERO, bool CHECK_NAN>
__device__ __forceinline__ void heap_stage(const KArgs& a, const unsigned char* stage, int cnt,
                                           int t0, ACC (&acc)[KMAX], uint32_t lane_off,
                                           const unsigned char* xrow, int64_t row, bool live) {
  using Node = HeapNode<XT>;
  const int D = a.depth;
  const int NI = (1 << D) - 1;
  const int NL = 1 << D;
  const int T = a.n_trees;
  const int64_t stride = a.tree_stride;
  const bool want_leaf = a.kind == TI_OUTPUT_LEAF;
  const uint32_t col_limit = (uint32_t)a.n_cols * (uint32_t)sizeof(XT);
  for (int j = 0; j < cnt; j += kTilp) {
    const Node* tp[kTilp];
#pragma unroll
    for (int q = 0; q < kTilp; ++q) {
      const int tq = (j + q) < cnt ? (j + q) : (cnt - 1);
      tp[q] = reinterpret_cast<const Node*>(stage + (int64_t)tq * stride);
    }
    uint32_t idx[kTilp];
#pragma unroll
    for (int q = 0; q < kTilp; ++q) idx[q] = 0u;
    for (int l = 0; l < D; ++l) {
      XT thr[kTilp];
      uint32_t meta[kTilp];
#pragma unroll
      for (int q = 0; q < kTilp; ++q) load_node(tp[q] + idx[q], thr[q], meta[q]);
      XT x[kTilp];
#pragma unroll
      for (int q = 0; q < kTilp; ++q) {
        const uint32_t off = meta[q] & kMetaFeatMask;
        if (FEAT_LDS) {
          x[q] = lds_at<XT>(off | lane_off);
        } else {
          x[q] = off < col_limit ? zero_map(*reinterpret_cast<const XT*>(xrow + off),
                                            a.lgb_zero_map)
                                 : nan_value<XT>();
        }
      }
#pragma unroll
      for (int q = 0; q < kTilp; ++q)
        idx[q] = 2u * idx[q] + (go_left<ZERO, CHECK_NAN>(x[q], thr[q], meta[q]) ? 1u : 2u);
    }
#pragma unroll
    for (int q = 0; q < kTilp; ++q) {
      if (j + q < cnt) {
        const int leaf = (int)idx[q] - NI;
        const int t = t0 + j + q;
        if (want_leaf) {
          if (live) static_cast<int32_t*>(a.out)[row * T + t] = a.heap_leaf_ids[(int64_t)t * NL + leaf];
        } else {
          const ACC* lv = reinterpret_cast<const ACC*>(tp[q] + NI);
          add_leaf<ACC, KMAX>(acc, lv, leaf, a.leaf_width, a.tree_group[t]);
        }
      }
    }
  }
}

template <typename XT, typename ACC, int KMAX, bool FEAT_LDS, bool ZERO>
__global__ void __launch_bounds__(512) heap_predict_kernel(const KArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int R = blockDim.x;
  const int tid = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * R;
  const int64_t row = row0 + tid;
  const bool live = row < a.n_rows;
  const size_t feat_bytes = FEAT_LDS ? align16((size_t)a.n_features * R * sizeof(XT)) : 0;
  volatile int* flag = reinterpret_cast<volatile int*>(smem + feat_bytes);
  unsigned char* stage = smem + feat_bytes + 16;
  const unsigned char* xrow = reinterpret_cast<const unsigned char*>(
      static_cast<const XT*>(a.X) + (live ? row : a.n_rows - 1) * a.row_stride);
  const uint32_t lane_off = (uint32_t)tid * (uint32_t)sizeof(XT);
  // without an LDS image the NaN path is always taken
  const bool tile_nan =
      FEAT_LDS ? stage_features<XT>(reinterpret_cast<XT*>(smem), flag, a, row0, R, tid) : true;
  const int T = a.n_trees;
  const int S = a.stage_trees;
  const int64_t stride = a.tree_stride;

  ACC acc[KMAX];
  init_acc(acc, a);

  // stage k covers trees [k*S, min(T, (k+1)*S)); the last stage re-prefetches
  // itself so the loop body has no conditional register traffic
  const int last0 = ((T - 1) / S) * S;
  u32x4 pf[kPf];
  prefetch_stage(pf, reinterpret_cast<const u32x4*>(a.trees),
                 (int)(((int64_t)(T < S ? T : S) * stride) >> 4), tid, R);
  for (int t0 = 0; t0 < T; t0 += S) {
    const int cnt = (T - t0) < S ? (T - t0) : S;
    __syncthreads();   // previous stage fully consumed (first pass: features staged)
    commit_stage(pf, reinterpret_cast<u32x4*>(stage), (int)(((int64_t)cnt * stride) >> 4), tid, R);
    __syncthreads();
    {                  // next stage in flight while this one is walked
      const int tn = t0 + S <= last0 ? t0 + S : last0;
      const int cn = (T - tn) < S ? (T - tn) : S;
      prefetch_stage(pf, reinterpret_cast<const u32x4*>(a.trees + (int64_t)tn * stride),
                     (int)(((int64_t)cn * stride) >> 4), tid, R);
    }
    if (tile_nan)
      heap_stage<XT, ACC, KMAX, FEAT_LDS, ZERO, true>(a, stage, cnt, t0, acc, lane_off, xrow, row, live);
    else
      heap_stage<XT, ACC, KMAX, FEAT_LDS, ZERO, false>(a, stage, cnt, t0, acc, lane_off, xrow, row, live);
  }
  if (!live || a.kind == TI_OUTPUT_LEAF) return;
  finish_row<ACC, KMAX>(acc, a, row);
}

// ------------------------------------------------------- binned heap kernel
// Rank binning.  For feature f let u_f[0] < ... < u_f[m-1] be the distinct
// canonical thresholds (float32 view: round_down_f32(t); float64 view: t) of
// all numerical splits on f.  A value x gets the bin b(x) = 1 + #{i : u_f[i] < x}
// and the split on threshold u_f[k] gets the rank k + 1, so
//     x <= u_f[k]   <=>   b(x) <= k + 1
// for every non-NaN x, exactly.  NaN gets the code kBinNan (the largest
// value of the bin width) and takes the node's NaN-left bit; a NaN threshold
// (xgboost's t = -inf) has rank 0 (never left); a padding node has rank
// 0xFFFF (always left, NaN included).  Bins are u16 (<= 65,533 thresholds
// per feature) or u8 (<= 253), so the tile's feature image shrinks 2-4x and
// more workgroups fit a CU -- which is what hides the LDS latency of the walk.
//
// The bin image in LDS is [word][R] of u32, each word packing P = 4/width
// features of one row: feature f of lane l sits at byte
//     (f / P) * R * 4 + l * 4 + (f % P) * width,
// so the lanes of a read hit 32 distinct banks whatever feature each tests.
// A binned heap node is one u32: bits 0..14 that byte offset minus the lane
// part, bit 15 NaN-left, bits 16..31 the rank.  With 512-row tiles the offset
// is word * 2048 + the byte of the word (bits 0, 1, 11..14) and the lane part
// is tid * 4 (bits 2..10), so bits 3..10 are free in the image: they hold the
// node's own heap index i (8 i = the byte offset of its children pair in the
// record), which the fixed-layout walk (bheap_fix_kernel) uses as the pair
// address.  a.bin_mask selects the offset bits (kBNodeOffMask512 then,
// kBNodeOffMask for smaller tiles, whose images carry no index).
constexpr uint32_t kBNodeNanLeft = 0x8000u;
constexpr uint32_t kBNodeOffMask = 0x7FFFu;
constexpr uint32_t kBNodeOffMask512 = 0x7803u;
constexpr uint32_t kBNodePairMask = 0x7F8u;

template <bool B16> struct BinTraits;
template <> struct BinTraits<true> { static constexpr int P = 2; static constexpr uint32_t kNan = 0xFFFFu; };
template <> struct BinTraits<false> { static constexpr int P = 4; static constexpr uint32_t kNan = 0xFFu; };

template <bool B16, bool CHECK_NAN>
__device__ __forceinline__ bool bin_left(uint32_t b, uint32_t nd) {
  bool left = b <= (nd >> 16);
  if (CHECK_NAN) left = left || (b == BinTraits<B16>::kNan && (nd & kBNodeNanLeft) != 0u);
  return left;
}

template <bool B16>
__device__ __forceinline__ uint32_t lds_bin(uint32_t byte_addr) {
  if (B16)
    return *reinterpret_cast<const __attribute__((address_space(3))) uint16_t*>(
        static_cast<uintptr_t>(byte_addr));
  return *reinterpret_cast<const __attribute__((address_space(3))) uint8_t*>(
      static_cast<uintptr_t>(byte_addr));
}

__device__ __forceinline__ uint32_t kpow5(int h) {
  uint32_t p = 1u;
  for (int i = 0; i < h; ++i) p *= 5u;
  return p;
}

// b[q] = 1 + #{u in U_f : u < x[q]} for Q consecutive features f0 + q (the
// last feature repeated past F; NaN gives an unspecified b, the caller codes
// it).  Two table forms (host: eytzinger_tables / kary_tables):
//  * Eytzinger: 2^L entries per feature, node k's children 2k and 2k+1,
//    +inf padded: L dependent 4- or 8-byte gathers;
//  * 5-ary (float32 view, a.bin_kary = H > 0): node j holds 4 sorted keys in
//    16 B, children 5j+1 .. 5j+5; after H levels j - (5^H - 1)/4 is the
//    count: H dependent 16-byte gathers (C2: 6 instead of 13).
// Q independent chains per lane hide the L2 latency of each level.
template <typename XT, int Q>
__device__ __forceinline__ void rank_search(const KArgs& a, const XT (&x)[Q], int f0,
                                            uint32_t (&b)[Q]) {
  const int F = a.n_features;
  uint32_t tq[Q], k[Q];
  if (sizeof(XT) == 4 && a.bin_kary > 0) {
    typedef float f4_t __attribute__((ext_vector_type(4)));
    const f4_t* t4 = reinterpret_cast<const f4_t*>(a.bin_tbl);
    const uint32_t nn = (kpow5(a.bin_kary) - 1u) / 4u;   // nodes per feature
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      tq[q] = (uint32_t)(f0 + q < F ? f0 + q : F - 1) * nn;
      k[q] = 0u;
    }
    for (int s = 0; s < a.bin_kary; ++s) {
      f4_t e[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q) e[q] = t4[tq[q] + k[q]];
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const XT xv = x[q];
        const uint32_t c = (e[q].x < xv ? 1u : 0u) + (e[q].y < xv ? 1u : 0u) +
                           (e[q].z < xv ? 1u : 0u) + (e[q].w < xv ? 1u : 0u);
        k[q] = 5u * k[q] + 1u + c;
      }
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) b[q] = 1u + k[q] - nn;
  } else {
    const XT* tbl = static_cast<const XT*>(a.bin_tbl);
    const uint32_t tsz = 1u << a.bin_L;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      tq[q] = (uint32_t)(f0 + q < F ? f0 + q : F - 1) * tsz;   // element offset, not a pointer
      k[q] = 1u;
    }
    for (int s = 0; s < a.bin_L; ++s) {
      XT e[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q) e[q] = tbl[tq[q] + k[q]];
#pragma unroll
      for (int q = 0; q < Q; ++q) k[q] = 2u * k[q] + (e[q] < x[q] ? 1u : 0u);
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) b[q] = 1u + k[q] - tsz;
  }
}

// Bin the tile's rows into the LDS bin image (at LDS address 0).  Columns go
// through `temp` (the tree-stage area, free at this point) bin_chunk at a
// time: a coalesced copy into [c][R], then every lane searches its own row's
// values (rank_search), Q features at once for Q independent load chains.
// Returns (uniformly) whether a live row of the tile holds a NaN.  Ends in a
// barrier.
template <typename XT, bool B16, int Q = TI_BIN_Q>
__device__ __forceinline__ bool stage_bins(volatile int* flag, XT* temp, const KArgs& a,
                                           int64_t row0, int R, int tid) {
  using BT = BinTraits<B16>;
  constexpr int P = BT::P;
  static_assert(Q % P == 0, "features searched at once: a multiple of the bins per word");
  const XT* X = static_cast<const XT*>(a.X);
  const int F = a.n_features;
  const int C = a.n_cols;
  const int64_t left_rows = a.n_rows - row0;
  const int rows_here = left_rows < R ? (int)left_rows : R;
  const bool vec_ok = ((reinterpret_cast<uintptr_t>(X) | (uintptr_t)(a.row_stride * sizeof(XT))) & 15) == 0;
  bool has_nan = false;
  if (tid == 0) *flag = 0;
  for (int f0 = 0; f0 < F; f0 += a.bin_chunk) {
    const int kc = (F - f0) < a.bin_chunk ? (F - f0) : a.bin_chunk;
    __syncthreads();   // temp is free (the previous chunk is searched)
    constexpr int V = 16 / sizeof(XT);   // elements per 16-byte load
    const bool vec = vec_ok && (f0 % V) == 0 && (kc % V) == 0 && f0 + kc <= C;
    const uint32_t n = (uint32_t)rows_here * (uint32_t)kc;
    const uint32_t ukc = (uint32_t)kc;
    if (vec) {
      // 16 bytes per lane (the row segments are 16-byte aligned): a quarter
      // (float) or half (double) of the load instructions of the loop below
      typedef XT xv_t __attribute__((ext_vector_type(V)));
      const uint32_t kv = ukc / V;
      const uint32_t nv = (uint32_t)rows_here * kv;
      for (uint32_t e = tid; e < nv; e += R) {
        const uint32_t r = e / kv;
        const uint32_t cv = e - r * kv;
        const xv_t v = *reinterpret_cast<const xv_t*>(X + (row0 + r) * a.row_stride + f0 + cv * V);
#pragma unroll
        for (int j = 0; j < V; ++j) temp[(cv * V + j) * R + r] = zero_map(v[j], a.lgb_zero_map);
      }
    }
    for (uint32_t e = vec ? n : tid; e < n; e += R) {
      const uint32_t r = e / ukc;
      const uint32_t c = e - r * ukc;
      const int f = f0 + (int)c;
      const XT v = f < C ? X[(row0 + r) * a.row_stride + f] : nan_value<XT>();
      temp[c * R + r] = zero_map(v, a.lgb_zero_map);
    }
    __syncthreads();
    for (int c = 0; c < kc; c += Q) {
      XT x[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q) x[q] = temp[(c + q < kc ? c + q : kc - 1) * R + tid];
      uint32_t b[Q];
      rank_search<XT, Q>(a, x, f0 + c, b);
      uint32_t w[Q / P];
#pragma unroll
      for (int j = 0; j < Q / P; ++j) w[j] = 0u;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const bool nan = x[q] != x[q];
        has_nan |= nan && (c + q < kc);
        w[q / P] |= (nan ? BT::kNan : b[q]) << ((q % P) * (32 / P));
      }
#pragma unroll
      for (int j = 0; j < Q / P; ++j) {
        const int word = (f0 + c) / P + j;
        if (c + j * P < kc) {
          __attribute__((address_space(3))) uint32_t* dst =
              reinterpret_cast<__attribute__((address_space(3))) uint32_t*>(
                  static_cast<uintptr_t>((uint32_t)(word * R + tid) * 4u));
          *dst = w[j];
        }
      }
    }
  }
  if (has_nan && tid < rows_here) *flag = 1;
  __syncthreads();
  return *flag != 0;
}

// Walk one LDS stage of binned complete trees.  A tree record is 2^D u32
// entries (1-based heap: node i has children 2i and 2i+1; entry 0 unused),
// then 2^D * leaf_width leaves (ACC).  At each level a lane issues the bin
// read of its current node's feature AND the read of the node's two children
// (one 8-byte word) together, so a level costs one LDS round trip, not two.
template <typename ACC, int KMAX, bool B16, bool CHECK_NAN>
__device__ __forceinline__ void bheap_stage(const KArgs& a, const unsigned char* stage, int cnt,
                                            int t0, ACC (&acc)[KMAX], uint32_t lane_off,
                                            int64_t row, bool live) {
  const int D = a.depth;
  const int NE = 1 << D;
  const int T = a.n_trees;
  const int64_t stride = a.tree_stride;
  const bool want_leaf = a.kind == TI_OUTPUT_LEAF;
  for (int j = 0; j < cnt; j += kBTilp) {
    const uint32_t* tp[kBTilp];
    uint32_t idx[kBTilp], nd[kBTilp];
#pragma unroll
    for (int q = 0; q < kBTilp; ++q) {
      const int tq = (j + q) < cnt ? (j + q) : (cnt - 1);
      tp[q] = reinterpret_cast<const uint32_t*>(stage + (int64_t)tq * stride);
      idx[q] = 1u;
      nd[q] = tp[q][1];   // the root: one broadcast read
    }
    // D levels: at the last one the children pair is two leaves (entries
    // [2^D, 2^(D+1)) are the leaf slots), so with float leaves of width 1 the
    // selected word is the leaf value itself -- no separate leaf read
    for (int l = 0; l < D; ++l) {
      uint32_t b[kBTilp];
      uint2 pr[kBTilp];
#pragma unroll
      for (int q = 0; q < kBTilp; ++q) {
        b[q] = lds_bin<B16>((nd[q] & a.bin_mask) | lane_off);
        pr[q] = *reinterpret_cast<const uint2*>(tp[q] + 2u * idx[q]);
      }
#pragma unroll
      for (int q = 0; q < kBTilp; ++q) {
#if TI_ASM_STEP == 2
        if (!CHECK_NAN) {
          uint64_t m;
          asm("v_cmp_lt_u32_sdwa %2, %0, %3 src0_sel:WORD_1 src1_sel:DWORD\n\t"
              "v_cndmask_b32_e64 %0, %4, %5, %2\n\t"
              "v_addc_co_u32_e64 %1, %2, %1, %1, %2"
              : "+v"(nd[q]), "+v"(idx[q]), "=&s"(m) : "v"(b[q]), "v"(pr[q].x), "v"(pr[q].y));
          continue;
        }
#elif TI_ASM_STEP
        if (!CHECK_NAN) {
          // right = rank < bin (SDWA compare on the node's high half), then the
          // child select and idx = 2 idx + right as one carry-in add: 3 VALU
          asm("v_cmp_lt_u32_sdwa vcc, %0, %2 src0_sel:WORD_1 src1_sel:DWORD\n\t"
              "v_cndmask_b32 %0, %3, %4, vcc\n\t"
              "v_addc_co_u32 %1, vcc, %1, %1, vcc"
              : "+v"(nd[q]), "+v"(idx[q]) : "v"(b[q]), "v"(pr[q].x), "v"(pr[q].y)
              : "vcc");
          continue;
        } else {
          // NaN tiles: right = (rank < bin) && !(bin == NaN code && NaN-left),
          // NaN-left being bit 15 = the sign of the node's low half as i16.
          // 5 VALU (the compiler's form: 9) and two SALU mask ops.
          uint64_t mn, ml;
          asm("v_cmp_lt_u32_sdwa vcc, %0, %4 src0_sel:WORD_1 src1_sel:DWORD\n\t"
              "v_cmp_eq_u32_e64 %2, %7, %4\n\t"
              "v_cmp_gt_i16_e64 %3, 0, %0\n\t"
              "s_and_b64 %2, %2, %3\n\t"
              "s_andn2_b64 vcc, vcc, %2\n\t"
              "v_cndmask_b32 %0, %5, %6, vcc\n\t"
              "v_addc_co_u32 %1, vcc, %1, %1, vcc"
              : "+v"(nd[q]), "+v"(idx[q]), "=&s"(mn), "=&s"(ml)
              : "v"(b[q]), "v"(pr[q].x), "v"(pr[q].y), "s"(BinTraits<B16>::kNan)
              : "vcc", "scc");
          continue;
        }
#endif
        const bool right = !bin_left<B16, CHECK_NAN>(b[q], nd[q]);
        idx[q] = idx[q] + idx[q] + (uint32_t)right;
        nd[q] = right ? pr[q].y : pr[q].x;
      }
    }
#pragma unroll
    for (int q = 0; q < kBTilp; ++q) {
      if (j + q < cnt) {
        const int leaf = (int)idx[q] - NE;
        const int t = t0 + j + q;
        if (want_leaf) {
          if (live) static_cast<int32_t*>(a.out)[row * T + t] = a.heap_leaf_ids[(int64_t)t * NE + leaf];
        } else if (sizeof(ACC) == 4 && a.leaf_width == 1) {
          const ACC v = __uint_as_float(nd[q]);   // the leaf the last level selected
          add_leaf<ACC, KMAX>(acc, &v, 0, 1, a.tree_group[t]);
        } else {
          const ACC* lv = reinterpret_cast<const ACC*>(tp[q] + NE);
          add_leaf<ACC, KMAX>(acc, lv, leaf, a.leaf_width, a.tree_group[t]);
        }
      }
    }
  }
}

template <int PF>
__device__ __forceinline__ void prefetch_n(u32x4 (&pf)[PF], const u32x4* __restrict__ src,
                                           int n16, int tid, int R) {
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    const int i = tid + u * R;
    pf[u] = src[i < n16 ? i : n16 - 1];
  }
}
template <int PF>
__device__ __forceinline__ void commit_n(const u32x4 (&pf)[PF], u32x4* __restrict__ dst, int n16,
                                         int tid, int R) {
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    const int i = tid + u * R;
    if (i < n16) dst[i] = pf[u];
  }
}

// Layout 9's stage copies: as prefetch_n / commit_n, but the loads address
// the uniform base with a 32-bit byte offset (the scalar-base form of
// global_load: an index clamp and a shift each) and the commit writes every
// word unconditionally (a clamped lane stores the last word's own value
// again: no compare and branch per store).  C3 5.41 -> 5.34 ms; the same
// copies measured about 1 % slower on C2 and C4, which keep the others
// (profiles/r2_copy_sweep.jsonl).
template <int PF>
__device__ __forceinline__ void prefetch_u(u32x4 (&pf)[PF], const u32x4* __restrict__ src,
                                           int n16, int tid, int R) {
  const unsigned char* base = reinterpret_cast<const unsigned char*>(src);
  const uint32_t last = (uint32_t)n16 - 1u;
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    const uint32_t i = (uint32_t)tid + (uint32_t)(u * R);
    pf[u] = *reinterpret_cast<const u32x4*>(base + (i < last ? i : last) * 16u);
  }
}
template <int PF>
__device__ __forceinline__ void commit_u(const u32x4 (&pf)[PF], u32x4* __restrict__ dst, int n16,
                                         int tid, int R) {
  const uint32_t last = (uint32_t)n16 - 1u;
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    const uint32_t i = (uint32_t)tid + (uint32_t)(u * R);
    dst[i < last ? i : last] = pf[u];
  }
}

// LDS: [bin image (bin_words * R u32)] [flag word] ... [stage area at
// stage_off: S tree records, also the binning temp].
template <typename XT, typename ACC, int KMAX, bool B16, int PF>
__global__ void __launch_bounds__(512) bheap_predict_kernel(const KArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int R = blockDim.x;
  const int tid = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * R;
  const int64_t row = row0 + tid;
  const bool live = row < a.n_rows;
  volatile int* flag = reinterpret_cast<volatile int*>(smem + (size_t)a.bin_words * R * 4);
  unsigned char* stage = smem + a.stage_off;
  const uint32_t lane_off = (uint32_t)tid * 4u;
  const int T = a.n_trees;
  const int S = a.stage_trees;
  const int64_t stride = a.tree_stride;
  // first stage in flight while the tile is binned
  u32x4 pf[PF];
  prefetch_n<PF>(pf, reinterpret_cast<const u32x4*>(a.trees),
                 (int)(((int64_t)(T < S ? T : S) * stride) >> 4), tid, R);
  const bool tile_nan = stage_bins<XT, B16>(flag, reinterpret_cast<XT*>(stage), a, row0, R, tid);

  ACC acc[KMAX];
  init_acc(acc, a);
  const int last0 = ((T - 1) / S) * S;
  for (int t0 = 0; t0 < T; t0 += S) {
    const int cnt = (T - t0) < S ? (T - t0) : S;
    __syncthreads();
    commit_n<PF>(pf, reinterpret_cast<u32x4*>(stage), (int)(((int64_t)cnt * stride) >> 4), tid, R);
    __syncthreads();
    {
      const int tn = t0 + S <= last0 ? t0 + S : last0;
      const int cn = (T - tn) < S ? (T - tn) : S;
      prefetch_n<PF>(pf, reinterpret_cast<const u32x4*>(a.trees + (int64_t)tn * stride),
                     (int)(((int64_t)cn * stride) >> 4), tid, R);
    }
    if (tile_nan)
      bheap_stage<ACC, KMAX, B16, true>(a, stage, cnt, t0, acc, lane_off, row, live);
    else
      bheap_stage<ACC, KMAX, B16, false>(a, stage, cnt, t0, acc, lane_off, row, live);
  }
  if (!live || a.kind == TI_OUTPUT_LEAF) return;
  finish_row<ACC, KMAX>(acc, a, row);
}

// ---- binned heap, fixed layout (C2: depth 8, scalar float leaves) ---------
// The same walk with compile-time LDS addresses.  A tile is 512 rows; the LDS
// is [bin image (<= 14 words x 2 KB)][flag @ kFixFlag][stage @ kFixStage: NG
// groups of 4 tree records of 2 KB].  Tree q of group g sits at the constant
// kFixStage + (4 g + q) * 2048, so the children pair of the current node is
// read at (nd & kBNodePairMask) + that constant (the node word carries its own
// heap index in bits 3..10, pack_bheap): no index register and no address
// arithmetic beyond one v_and_b32 with a literal.  A level is then
//   v_and_or_b32 (bin address), v_and_b32 (pair address),
//   ds_read_u16 / ds_read_u8 + ds_read_b64 (issued together),
//   v_cmp_lt_u32_sdwa (rank < bin), v_cndmask_b32 (next node word)
// = 4 VALU instead of 5, and the v_lshl_add / v_addc pair that the index
// cost is gone (scripts/micro/valu_rate.hip: 6.6 vs 9.6 cycles per step per
// SIMD at 8 waves).  At the last level the pair holds two leaves, so the
// selected word is the leaf value.  Leaves are added in tree order, so the
// float32 sums are xgboost's.  The host takes this kernel for float32
// accumulators, one leaf value per leaf, depth-8 images of 512-row tiles and
// <= 14 bin words; leaf ids (TI_OUTPUT_LEAF) keep bheap_predict_kernel.
constexpr uint32_t kFixFlag = 28672u;
constexpr uint32_t kFixStage = 30720u;
constexpr int kFixRows = 512;
constexpr int kFixTree = 2048;   // 256 node words + 256 float leaves

__device__ __forceinline__ uint2 lds_u2c(uint32_t byte_addr) {
  const uint64_t v = *reinterpret_cast<const __attribute__((address_space(3))) uint64_t*>(
      static_cast<uintptr_t>(byte_addr));
  return make_uint2((uint32_t)v, (uint32_t)(v >> 32));
}
__device__ __forceinline__ uint32_t lds_u32(uint32_t byte_addr) {
  return *reinterpret_cast<const __attribute__((address_space(3))) uint32_t*>(
      static_cast<uintptr_t>(byte_addr));
}

#ifndef TI_FIX_SROOT
#define TI_FIX_SROOT 1
#endif
// SROOT: the root and its children pair are the same for every lane, so words
// 0..3 of each tree's image come as scalar loads from global memory, issued
// between the two barriers of the stage commit (whose LDS wait covers their
// latency; a scalar load still in flight would make every LDS wait of the walk
// wait for it), and level 0 is the bin read, a compare against the scalar rank
// and a select between two scalars: no pair read from LDS.  C2 0.787 -> 0.775
// ms (profiles/r3_c2_sroot_ab.jsonl); level 1's pair selected from the four
// scalars of level 2 by level 0's decision was 5 % slower (its VALU selects
// cost more than the LDS read they replace).
typedef const __attribute__((address_space(4))) u32x4 fix_cu4_t;
template <int NG>
__device__ __forceinline__ void fix_tops(const KArgs& a, int t0, u32x4 (&top)[4 * NG]) {
  fix_cu4_t* timg = reinterpret_cast<fix_cu4_t*>(reinterpret_cast<uintptr_t>(a.trees));
#pragma unroll
  for (int i = 0; i < 4 * NG; ++i) top[i] = timg[min(t0 + i, a.n_trees - 1) * (kFixTree / 16)];
}
template <bool B16, bool CHECK_NAN>
__device__ __forceinline__ void fix_step(uint32_t& nd, uint32_t b, uint2 pr) {
  if (!CHECK_NAN) {
    asm("v_cmp_lt_u32_sdwa vcc, %0, %1 src0_sel:WORD_1 src1_sel:DWORD\n\t"
        "v_cndmask_b32 %0, %2, %3, vcc"
        : "+v"(nd) : "v"(b), "v"(pr.x), "v"(pr.y) : "vcc");
  } else {
    // right = (rank < bin) && !(bin == NaN code && NaN-left (bit 15))
    uint64_t mn, ml;
    asm("v_cmp_lt_u32_sdwa vcc, %0, %3 src0_sel:WORD_1 src1_sel:DWORD\n\t"
        "v_cmp_eq_u32_e64 %1, %6, %3\n\t"
        "v_cmp_gt_i16_e64 %2, 0, %0\n\t"
        "s_and_b64 %1, %1, %2\n\t"
        "s_andn2_b64 vcc, vcc, %1\n\t"
        "v_cndmask_b32 %0, %4, %5, vcc"
        : "+v"(nd), "=&s"(mn), "=&s"(ml)
        : "v"(b), "v"(pr.x), "v"(pr.y), "s"(BinTraits<B16>::kNan)
        : "vcc", "scc");
  }
}
template <int KMAX, bool B16, bool CHECK_NAN, int NG>
__device__ __forceinline__ void bheap_fix_stage(const KArgs& a, int cnt, int t0, float (&acc)[KMAX],
                                                uint32_t lane_off, const u32x4 (&top)[4 * NG]) {
  const uint32_t bmask = a.bin_mask;
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    if (g * 4 >= cnt) break;   // uniform: the last stage may be short
    uint32_t nd[4];
#if TI_FIX_SROOT
    {
      uint32_t b0[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) b0[q] = lds_bin<B16>((top[g * 4 + q].y & bmask) | lane_off);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const u32x4 tp = top[g * 4 + q];
        // v_cmp against the scalar rank, two v_mov and a v_cndmask (with vcc
        // as the mask, gfx9's constant bus takes no SGPR source besides it)
        bool right = (tp.y >> 16) < b0[q];
        if (CHECK_NAN && (tp.y & 0x8000u)) right = right && b0[q] != BinTraits<B16>::kNan;
        nd[q] = right ? tp.w : tp.z;
      }
    }
    constexpr int l_first = 1;
#else
    (void)top;
#pragma unroll
    for (int q = 0; q < 4; ++q) nd[q] = lds_u32(kFixStage + (uint32_t)((g * 4 + q) * kFixTree) + 4u);
    constexpr int l_first = 0;
#endif
#pragma unroll
    for (int l = l_first; l < 8; ++l) {
      uint32_t b[4];
      uint2 pr[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        b[q] = lds_bin<B16>((nd[q] & bmask) | lane_off);
        pr[q] = lds_u2c((nd[q] & kBNodePairMask) + (kFixStage + (uint32_t)((g * 4 + q) * kFixTree)));
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) fix_step<B16, CHECK_NAN>(nd[q], b[q], pr[q]);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int t = t0 + g * 4 + q;
      if (g * 4 + q < cnt) {
        const float v = __uint_as_float(nd[q]);   // the leaf the last level selected
        add_leaf<float, KMAX>(acc, &v, 0, 1, KMAX == 1 ? 0 : a.tree_group[t]);
      }
    }
  }
}

template <typename XT, int KMAX, bool B16, int NG>
__global__ void __launch_bounds__(512) bheap_fix_kernel(const KArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int R = kFixRows;
  constexpr int S = 4 * NG;   // trees per stage
  const int tid = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * R;
  const int64_t row = row0 + tid;
  const bool live = row < a.n_rows;
  volatile int* flag = reinterpret_cast<volatile int*>(smem + kFixFlag);
  u32x4* stage = reinterpret_cast<u32x4*>(smem + kFixStage);
  const uint32_t lane_off = (uint32_t)tid * 4u;
  const int T = a.n_trees;
  constexpr int n16 = S * kFixTree / 16;   // 16-byte words per stage: NG per thread
  static_assert(n16 == NG * R, "one 16-byte word per thread and group");
  const u32x4* src = reinterpret_cast<const u32x4*>(a.trees);
  const int n16_all = (int)(((int64_t)T * kFixTree) >> 4);
  // first stage in flight while the tile is binned (a clamped lane re-reads
  // the forest's last word; its stage slot then holds a word no tree reads)
  u32x4 pf[NG];
#pragma unroll
  for (int u = 0; u < NG; ++u) {
    const int i = tid + u * R;
    pf[u] = src[i < n16_all ? i : n16_all - 1];
  }
  const bool tile_nan = stage_bins<XT, B16, 4 * NG>(
      flag, reinterpret_cast<XT*>(smem + kFixStage), a, row0, R, tid);
  float acc[KMAX];
  init_acc(acc, a);
  u32x4 top[4 * NG] = {};
  for (int t0 = 0; t0 < T; t0 += S) {
    const int cnt = (T - t0) < S ? (T - t0) : S;
    __syncthreads();
#if TI_FIX_SROOT
    fix_tops<NG>(a, t0, top);
#endif
#pragma unroll
    for (int u = 0; u < NG; ++u) stage[tid + u * R] = pf[u];
    __syncthreads();
    {
      const int base = (t0 + S) * (kFixTree / 16);
#pragma unroll
      for (int u = 0; u < NG; ++u) {
        const int i = base + tid + u * R;
        pf[u] = src[i < n16_all ? i : n16_all - 1];
      }
    }
    if (tile_nan)
      bheap_fix_stage<KMAX, B16, true, NG>(a, cnt, t0, acc, lane_off, top);
    else
      bheap_fix_stage<KMAX, B16, false, NG>(a, cnt, t0, acc, lane_off, top);
  }
  if (!live) return;
  finish_row<float, KMAX>(acc, a, row);
}

// ------------------------------------------------------------ explicit kernel
// Any tree shape; nodes stay in global memory (L2 / MALL).  meta bits 0..23
// hold the plain feature index.  Each lane walks kExpIlp trees at once with
// unconditional (clamped) node loads so the dependent L2 round trips of the
// trees overlap; finished trees keep their leaf code.
template <typename XT, typename ACC, int KMAX, bool FEAT_LDS, bool ZERO>
__global__ void __launch_bounds__(512) explicit_predict_kernel(const KArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int R = blockDim.x;
  const int tid = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * R;
  const int64_t row = row0 + tid;
  const bool live = row < a.n_rows;
  XT* feat = reinterpret_cast<XT*>(smem);
  const XT* xrow = static_cast<const XT*>(a.X) + (live ? row : a.n_rows - 1) * a.row_stride;
  if (FEAT_LDS) {
    volatile int* flag = reinterpret_cast<volatile int*>(
        smem + align16((size_t)a.n_features * R * sizeof(XT)));
    stage_features<XT>(feat, flag, a, row0, R, tid);   // ends in a barrier
  }
  const int T = a.n_trees;
  const bool want_leaf = a.kind == TI_OUTPUT_LEAF;
  int32_t* out_leaf = static_cast<int32_t*>(a.out);
  const ACC* leaves = static_cast<const ACC*>(a.leaves);

  ACC acc[KMAX];
  init_acc(acc, a);

  for (int t0 = 0; t0 < T; t0 += kExpIlp) {
    int64_t nb[kExpIlp];
    int32_t c[kExpIlp];
#pragma unroll
    for (int q = 0; q < kExpIlp; ++q) {
      const int tq = (t0 + q) < T ? (t0 + q) : (T - 1);
      nb[q] = a.node_base[tq];
      c[q] = a.root[tq];
    }
    for (;;) {
      u32x4 nd[kExpIlp];   // {thr32 bits, meta, left, right}; native vector stays in VGPRs
#pragma unroll
      for (int q = 0; q < kExpIlp; ++q)
        nd[q] = *reinterpret_cast<const u32x4*>(a.nodes + nb[q] + (c[q] < 0 ? 0 : c[q]));
      XT thr[kExpIlp];
#pragma unroll
      for (int q = 0; q < kExpIlp; ++q)
        thr[q] = sizeof(XT) == 4 ? (XT)__uint_as_float(nd[q].x)
                                 : (XT)a.thr64[nb[q] + (c[q] < 0 ? 0 : c[q])];
      bool active = false;
#pragma unroll
      for (int q = 0; q < kExpIlp; ++q) {
        const uint32_t f = nd[q].y & kMetaFeatMask;
        XT x;
        if (FEAT_LDS) {
          x = feat[f * R + tid];
        } else {
          x = (int)f < a.n_cols ? zero_map(xrow[f], a.lgb_zero_map) : nan_value<XT>();
        }
        bool l = go_left<ZERO>(x, thr[q], nd[q].y);
        if (a.cat_words != nullptr && (nd[q].y & kMetaCat))   // uniform test, then rare branch
          l = cat_left(a.cat_words + nd[q].x, (double)x);
        const int32_t next = l ? (int32_t)nd[q].z : (int32_t)nd[q].w;
        c[q] = c[q] < 0 ? c[q] : next;
        active |= c[q] >= 0;
      }
      if (__ballot(active) == 0) break;
    }
#pragma unroll
    for (int q = 0; q < kExpIlp; ++q) {
      const int t = t0 + q;
      if (t < T) {
        const int64_t lb = a.leaf_base[t];
        if (want_leaf) {
          if (live) out_leaf[row * T + t] = a.exp_leaf_ids[lb + (~c[q])];
        } else {
          add_leaf<ACC, KMAX>(acc, leaves + lb * a.leaf_width, ~c[q], a.leaf_width,
                              a.tree_group[t]);
        }
      }
    }
  }
  if (!live || want_leaf) return;
  finish_row<ACC, KMAX>(acc, a, row);
}

// ---- record explicit (layout 6) --------------------------------------------
// Deep / irregular trees (LightGBM leaf-wise C3, sklearn depth 16 C4).  What
// bounds a walk whose nodes come from L2 is the vector-memory pipe, not the
// ALU: the PMC pass of the binned explicit kernel (layout 4, 16-byte nodes,
// profiles/r2_c3_l4_pmc.json) has the TD busy ~93 % of the kernel and the TA
// ~77 %, i.e. the cost is the number of 64-byte requests a wave's gather
// makes (one per distinct sector within each group of lanes the TA takes per
// cycle: 4 lanes for 16-byte loads, 8 for 8-byte).  So this layout
//   * uses 8-byte records (twice the lanes per TA cycle, twice the nodes per
//     sector);
//   * masks the gathers of lanes already at a leaf (a finished lane makes no
//     request; a tree whose 64 lanes are all done costs the wave nothing);
//   * keeps the leaf value in the leaf's own record, so reaching the leaf is
//     the last gather of the tree (layout 4 gathers the value again).
// A tree is a block of slots: internal nodes [0, nint) breadth-first, then the
// leaves [nint, nslots).  Internal record:
//   x = rank << 16 | bin byte offset (lane-free part, even: u16 bins) | NaN-left
//   y = right slot << 16 | left slot
// Leaf record: the leaf value (ACC: float in x, or double in x:y) when leaves
// are scalars; leaf ids and vector leaves are found from the slot (leaf index =
// the tree's first leaf + slot - nint).  Split rule on bins:
//   right = (rank < b) ^ (b == kNan && NaN-left)
// LightGBM zero-missing forests (ZERO) bin as b2 = 2 b + (x == 0) with NaN =
// 0xFFFE and store rank2 = 2 rank + 1 (rank2 < b2 <=> rank < b, exactly) and
// the zero flip in x bit 2 (the bin offset's lane part, clear in the record):
//   right ^= (b2 odd) && zero-flip.
// A tile whose rows hold no NaN (and, for ZERO, no exact 0 after LightGBM's
// zero map) needs neither term: b2 is even there, so the step is the plain
// rank compare on x's high half for every forest (rx_next_fast, 2 VALU).
constexpr uint32_t kRxNanLeft = 1u;
constexpr uint32_t kRxZeroFlip = 4u;
constexpr uint32_t kRxOffMask = 0xFFFAu;   // the bin byte offset without the flag bits
// u8 bins (layout 9 when every feature has <= 254 distinct thresholds, <= 126
// with the zero rule; lightgbm max_bin = 255 models): four features per word,
// so the byte offset keeps bits 0-1 and the flags move into the lane part
// (bits 2 and 3, cleared before the lane offset is OR-ed in).  NaN is bin 0
// (the bins of values are 1 .. m + 1), which the rank compare sends left; a
// tile holding a NaN takes the slow step, which tests b == 0 first.
template <bool B8> struct RxBins {
  static constexpr uint32_t kNanLeft = 1u, kZeroFlip = 4u, kOffMask = 0xFFFAu;
  static constexpr uint32_t kLeaf = 0u;   // (the compact bottom is u8 only)
  template <bool ZERO> static constexpr uint32_t nan_code() { return ZERO ? 0xFFFEu : 0xFFFFu; }
  static constexpr int kPerWord = 2;
};
template <> struct RxBins<true> {
  static constexpr uint32_t kNanLeft = 4u, kZeroFlip = 8u, kOffMask = 0xFFF3u;
  // the compact bottom (t8explicit): a leaf's x carries kLeaf (bit 4, in the
  // lane part); kNodeMask clears the flags, the leaf bit, the rank (byte 2)
  // and the pair index (byte 3) from a bin address
  static constexpr uint32_t kLeaf = 16u, kNodeMask = 0xFFE3u;
  template <bool ZERO> static constexpr uint32_t nan_code() { return 0u; }
  static constexpr int kPerWord = 4;
};

// Slot loads are structured buffer loads: vindex = the slot (VGPR), soffset =
// the tree's first byte (wave-uniform SGPR), stride 8 in the resource, so the
// slot -> address step costs no VALU (buffer_load_dwordx2 ... idxen).
typedef int rx_rsrc_t __attribute__((ext_vector_type(4)));
typedef unsigned rx_u2_t __attribute__((ext_vector_type(2)));
__device__ rx_u2_t rx_struct_load(rx_rsrc_t rsrc, uint32_t vindex, uint32_t voffset,
                                  uint32_t soffset, int aux)
    __asm("llvm.amdgcn.struct.buffer.load.v2i32");

__device__ __forceinline__ rx_rsrc_t rx_make_rsrc(const void* base, uint32_t n_slots) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  rx_rsrc_t r;
  r.x = static_cast<int>(static_cast<uint32_t>(a));
  r.y = static_cast<int>(static_cast<uint32_t>(a >> 32) | (8u << 16));   // stride 8 B
  r.z = static_cast<int>(n_slots);                                         // records (slots)
  r.w = 0x00020000;                                                        // 32-bit data format
  return r;
}

// One split decision.  The fast form (tiles without NaN / exact zeros) is the
// rank compare of the record's high half with the bin and one SDWA select of
// the child from the two halves of y on the compare's mask: 2 VALU.  The bin
// comes straight from ds_read_u16 as a 16-bit value; the compare reads its low
// word (src1_sel:WORD_0), so no zero-extension is spent on it.  The slow form
// adds the zero flip and the NaN direction (rare tiles; compiler-scheduled).
__device__ __forceinline__ uint32_t rx_next_fast(uint32_t x, uint32_t y, uint16_t b) {
  uint32_t slot;
  asm("v_cmp_lt_u32_sdwa vcc, %1, %3 src0_sel:WORD_1 src1_sel:WORD_0\n\t"
      "v_cndmask_b32_sdwa %0, %2, %2, vcc src0_sel:WORD_0 src1_sel:WORD_1"
      : "=v"(slot) : "v"(x), "v"(y), "v"(b) : "vcc");
  return slot;
}
template <bool ZERO, bool B8 = false>
__device__ __forceinline__ uint32_t rx_next_slow(uint32_t x, uint32_t y, uint16_t b16) {
  using W = RxBins<B8>;
  constexpr uint32_t kNan = W::template nan_code<ZERO>();
  const uint32_t b = b16;
  bool right = (x >> 16) < b;
  if (ZERO) right = right != (((b & 1u) != 0u) && ((x & W::kZeroFlip) != 0u));
  if (b == kNan) right = (x & W::kNanLeft) == 0u;
  return right ? (y >> 16) : (y & 0xFFFFu);
}
template <bool ZERO, bool SLOW, bool B8 = false>
__device__ __forceinline__ uint32_t rx_next(uint32_t x, uint32_t y, uint16_t b) {
  return SLOW ? rx_next_slow<ZERO, B8>(x, y, b) : rx_next_fast(x, y, b);
}
__device__ __forceinline__ uint16_t lds_u16(uint32_t byte_addr) {
  return *reinterpret_cast<const __attribute__((address_space(3))) uint16_t*>(
      static_cast<uintptr_t>(byte_addr));
}
__device__ __forceinline__ uint16_t lds_u8(uint32_t byte_addr) {
  return *reinterpret_cast<const __attribute__((address_space(3))) uint8_t*>(
      static_cast<uintptr_t>(byte_addr));
}
template <bool B8>
__device__ __forceinline__ uint16_t lds_rxbin(uint32_t byte_addr) {
  return B8 ? lds_u8(byte_addr) : lds_u16(byte_addr);
}

// Bin the tile's rows (one lane per row, per-lane loads)
// into the u16 image of layouts 6 / 7: b = 1 + #{u < x}, NaN = 0xFFFF; with ZB
// (zero-missing forests) b2 = 2 b + (x == 0) and NaN = 0xFFFE.  Returns
// (uniformly) whether the tile needs the slow step: a NaN, or with ZB an
// exact 0.
#ifndef TI_RX_POSTSTEP
#define TI_RX_POSTSTEP 1   // layout 6: the group's loop test reads the lanes after the
                           // step, so no pass runs once every lane is at its leaf
#endif
#ifndef TI_RX_BINQ
#define TI_RX_BINQ 8   // features searched at once per lane (independent load chains;
                       // 16 measured slower on C3 and C4)
#endif
// Search Q consecutive features [f0, f0 + Q) of the lane's row (values x,
// NaN past the last feature) and store their packed u16 bins in the image
// (f0 even).  With ZB (zero-missing forests) b2 = 2 b + (x == 0), NaN 0xFFFE.
template <typename XT, bool ZB, bool KARY, int Q, bool SROOT = false, bool B8 = false>
__device__ __forceinline__ void rx_bin_group(const KArgs& a, const XT (&x)[Q], int f0, int R, int tid,
                                             bool& has_nan) {
  const int F = a.n_features;
  const uint32_t tsz = 1u << a.bin_L;
  uint32_t tq[Q], k[Q];
  if (KARY) {
    // 5-ary search tree: node j holds 4 sorted keys (16 B for the float32
    // view, 32 B for float64), its children are 5j+1 .. 5j+5; after H levels
    // j - (5^H - 1)/4 is the number of keys below x.  H gathers instead of L.
    typedef XT f4_t __attribute__((ext_vector_type(4)));
    const f4_t* t4 = reinterpret_cast<const f4_t*>(a.bin_tbl);
    const uint32_t nn = (kpow5(a.bin_kary) - 1u) / 4u;   // nodes per feature
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      tq[q] = (uint32_t)(f0 + q < F ? f0 + q : F - 1) * nn;
      k[q] = 0u;
    }
    int s0 = 0;
    if (SROOT) {   // the root, the same node for every lane, as a scalar load
      typedef const __attribute__((address_space(4))) f4_t cf4_t;
      cf4_t* s4 = reinterpret_cast<cf4_t*>(reinterpret_cast<uintptr_t>(a.bin_tbl));
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const f4_t e = s4[tq[q]];
        const XT xv = x[q];
        k[q] = 1u + (e.x < xv ? 1u : 0u) + (e.y < xv ? 1u : 0u) + (e.z < xv ? 1u : 0u) +
               (e.w < xv ? 1u : 0u);
      }
      s0 = 1;
    }
    for (int s = s0; s < a.bin_kary; ++s) {
      f4_t e[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q) e[q] = t4[tq[q] + k[q]];
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const XT xv = x[q];
        const uint32_t c = (e[q].x < xv ? 1u : 0u) + (e[q].y < xv ? 1u : 0u) +
                           (e[q].z < xv ? 1u : 0u) + (e[q].w < xv ? 1u : 0u);
        k[q] = 5u * k[q] + 1u + c;
      }
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) k[q] = k[q] - nn + tsz;   // as the Eytzinger end: b = 1 + k - tsz
  } else {
    const XT* tbl = static_cast<const XT*>(a.bin_tbl);
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      tq[q] = (uint32_t)(f0 + q < F ? f0 + q : F - 1) * tsz;   // element offset, not a pointer
      k[q] = 1u;
    }
    for (int s = 0; s < a.bin_L; ++s) {
      XT e[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q) e[q] = tbl[tq[q] + k[q]];
#pragma unroll
      for (int q = 0; q < Q; ++q) k[q] = 2u * k[q] + (e[q] < x[q] ? 1u : 0u);
    }
  }
  constexpr int P = RxBins<B8>::kPerWord;   // bins per 32-bit word (f0 % P == 0)
  constexpr uint32_t kNan = RxBins<B8>::template nan_code<ZB>();
  uint32_t w[Q / P];
#pragma unroll
  for (int j = 0; j < Q / P; ++j) w[j] = 0u;
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const bool nan = x[q] != x[q];
    const bool zero = ZB && x[q] == XT(0);
    has_nan |= (nan || zero) && (f0 + q < F);   // the tile needs the slow step
    uint32_t b = 1u + k[q] - tsz;
    if (ZB) b = nan ? kNan : 2u * b + (zero ? 1u : 0u);
    else b = nan ? kNan : b;
    w[q / P] |= b << ((q % P) * (32 / P));
  }
#pragma unroll
  for (int j = 0; j < Q / P; ++j) {
    const int word = f0 / P + j;
    if (word < a.bin_words) {
      __attribute__((address_space(3))) uint32_t* dst =
          reinterpret_cast<__attribute__((address_space(3))) uint32_t*>(
              static_cast<uintptr_t>((uint32_t)(word * R + tid) * 4u));
      *dst = w[j];
    }
  }
}

// Bin the tile's rows into the u16 image of layouts 6 to 9.  With a temp area
// (temp != nullptr: the stage area of layouts 7-9, free until the first stage
// is committed; a.bin_chunk columns of R rows) and 16-byte-aligned rows, the
// tile's X goes through it a chunk of columns at a time in coalesced 16-byte
// loads (a 64-lane load touches 8 lines), and each lane then reads its row's
// values from LDS; otherwise every lane loads its own row (a load touches 64
// lines: C3's 400-byte rows made that 0.57 ms of a 5.5 ms kernel).  Returns
// (uniformly) whether the tile needs the slow step: a NaN, or with ZB an
// exact 0.
// NT threads bin the R-row tile (NT = R, or 2R for the two-lanes-a-row walk:
// thread tid takes row tid mod R and every (NT / R)-th group of Q features).
template <typename XT, bool ZB, bool KARY = false, bool SROOT = false, bool B8 = false>
__device__ __forceinline__ bool rx_stage_bins_impl(volatile int* flag, XT* temp, const KArgs& a,
                                                   int64_t row0, int R, int tid_in, int NT) {
  constexpr int Q = TI_RX_BINQ;
  const int F = a.n_features;
  const int FC = F < a.n_cols ? F : a.n_cols;
  const int tid = tid_in & (R - 1);          // the row this thread bins (R: a power of two)
  const int H = NT / R, h = tid_in / R;      // feature groups h, h + H, h + 2H, ...
  const int64_t row = row0 + tid;
  const bool live = row < a.n_rows;
  const XT* X = static_cast<const XT*>(a.X);
  bool has_nan = false;
  if (tid_in == 0) *flag = 0;
  constexpr int V = 16 / sizeof(XT);   // elements per 16-byte load
  const bool tiled = temp != nullptr && a.bin_chunk >= Q && FC == F && (F % V) == 0 &&
                     ((reinterpret_cast<uintptr_t>(X) | (uintptr_t)(a.row_stride * sizeof(XT))) & 15) == 0;
  if (tiled) {
    typedef XT xv_t __attribute__((ext_vector_type(V)));
    const int64_t left = a.n_rows - row0;
    const uint32_t rows_here = left < R ? (uint32_t)left : (uint32_t)R;
    for (int f0 = 0; f0 < F; f0 += a.bin_chunk) {
      const int kc = (F - f0) < a.bin_chunk ? (F - f0) : a.bin_chunk;
      const uint32_t kv = (uint32_t)kc / V;
      __syncthreads();   // temp is free: the previous chunk is searched
      for (uint32_t e = tid_in; e < rows_here * kv; e += NT) {
        const uint32_t r = e / kv;
        const uint32_t cv = e - r * kv;
        const xv_t v = *reinterpret_cast<const xv_t*>(X + (row0 + r) * a.row_stride + f0 + cv * V);
#pragma unroll
        for (int j = 0; j < V; ++j) temp[(cv * V + j) * R + r] = zero_map(v[j], a.lgb_zero_map);
      }
      __syncthreads();
      for (int c = h * Q; c < kc; c += Q * H) {
        XT x[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) x[q] = c + q < kc ? temp[(c + q) * R + tid] : nan_value<XT>();
        rx_bin_group<XT, ZB, KARY, Q, SROOT, B8>(a, x, f0 + c, R, tid, has_nan);
      }
    }
  } else {
    const XT* xr = X + (live ? row : a.n_rows - 1) * a.row_stride;
    for (int f0 = h * Q; f0 < F; f0 += Q * H) {
      XT x[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int f = f0 + q < F ? f0 + q : F - 1;
        x[q] = f0 + q < FC ? zero_map(xr[f], a.lgb_zero_map) : nan_value<XT>();
      }
      rx_bin_group<XT, ZB, KARY, Q, SROOT, B8>(a, x, f0, R, tid, has_nan);
    }
  }
  __syncthreads();   // flag = 0 is visible before any lane sets it
  if (has_nan && live) *flag = 1;
  __syncthreads();
  return *flag != 0;
}

// Both views search the 5-ary tables when the host built them (a.bin_kary >
// 0: float32 16-byte nodes, float64 32-byte ones), else the Eytzinger tables.
// SROOT: the 5-ary root as a scalar load (layout 8: C4 2.17 -> 2.13 ms; on
// layout 9 it cost C3 0.7 %, profiles/r2_kary_root_sweep.jsonl)
template <typename XT, bool ZB, bool SROOT = false, bool B8 = false>
__device__ __forceinline__ bool rx_stage_bins(volatile int* flag, const KArgs& a, int64_t row0,
                                              int R, int tid, void* temp = nullptr, int NT = 0) {
  if (NT <= 0) NT = R;
  if (a.bin_kary > 0)
    return rx_stage_bins_impl<XT, ZB, true, SROOT, B8>(flag, static_cast<XT*>(temp), a, row0, R,
                                                       tid, NT);
  return rx_stage_bins_impl<XT, ZB, false, false, B8>(flag, static_cast<XT*>(temp), a, row0, R, tid,
                                                      NT);
}

// Per step every tree's bin read is issued first, then each tree's decision
// and its exec-masked gather: only lanes still inside the tree decide and
// gather, so a finished lane makes no request and keeps its record -- the
// leaf's value, read by the gather that reached it.  `in` comes from the slot
// at the start of the step (no lane-mask state is carried across iterations:
// the compiler would rebuild every mask in every branch); the loop runs one
// step past the group's last leaf.  A lane at its leaf reads its own column
// of bin word 0 instead of an address made of its record's value bits: the
// random addresses of finished lanes made 66 % of the LDS cycles bank
// conflicts (profiles/r2_c3_l6c_pmc.json).  VIS: scalar leaf values sit in
// the leaf records; otherwise the slot gives the leaf index.
template <typename ACC, int KMAX>
__device__ __forceinline__ void rx_leaves(const KArgs& a, ACC (&acc)[KMAX], int t, uint32_t slot,
                                          uint32_t ni, uint32_t rx, uint32_t ry, int64_t row,
                                          bool live, bool vis) {
  const int LW = a.leaf_width;
  if (vis) {
    ACC v;
    if (sizeof(ACC) == 8) v = (ACC)__hiloint2double((int)ry, (int)rx);
    else v = (ACC)__uint_as_float(rx);
    add_leaf<ACC, KMAX>(acc, &v, 0, 1, a.tree_group[t]);
    return;
  }
  // leaf ids / vector leaves: the leaf's index from its slot
  const int64_t li = a.leaf_base[t] + (int64_t)(slot - ni);
  if (a.kind == TI_OUTPUT_LEAF) {
    if (live) static_cast<int32_t*>(a.out)[row * a.n_trees + t] = a.exp_leaf_ids[li];
  } else {
    add_leaf<ACC, KMAX>(acc, static_cast<const ACC*>(a.leaves) + li * LW, 0, LW, a.tree_group[t]);
  }
}

typedef const __attribute__((address_space(4))) uint32_t rx_cu32;   // scalar-loaded tables

#ifndef TI_RX_ADDR2
#define TI_RX_ADDR2 1
#endif
// The bin address of a record step (layouts 6-9): (x & mask) | lane offset
// inside a tree, the lane's own column of word 0 at its leaf.  The empty asm keeps the
// compiler from rewriting the select as and / cndmask / or: v_and_or_b32 and
// one v_cndmask_b32, 2 VALU instead of 3.
template <bool B8 = false>
__device__ __forceinline__ uint32_t rx_bin_addr(uint32_t x, bool in, uint32_t lane_off) {
  uint32_t t = (x & RxBins<B8>::kOffMask) | lane_off;
#if TI_RX_ADDR2
  asm("" : "+v"(t));
#endif
  return in ? t : lane_off;
}

// The lockstep descent of a group of ILP trees from each lane's current slot
// (and the record gathered there) to its leaf.
template <bool ZERO, bool SLOW, int ILP>
__device__ __forceinline__ void rx_descend(const rx_rsrc_t rsrc, const uint32_t (&sb)[ILP],
                                           const uint32_t (&ni)[ILP], uint32_t (&slot)[ILP],
                                           rx_u2_t (&rec)[ILP], uint32_t lane_off) {
#if TI_RX_POSTSTEP
  bool in[ILP];
  bool any = false;
#pragma unroll
  for (int q = 0; q < ILP; ++q) {
    in[q] = slot[q] < ni[q];
    any |= in[q];
  }
  while (__ballot(any) != 0) {   // a lane of the group is still inside a tree
    uint32_t b[ILP];
#pragma unroll
    for (int q = 0; q < ILP; ++q)   // a lane at its leaf reads its own column of word 0
      b[q] = lds_u16(rx_bin_addr(rec[q].x, in[q], lane_off));
    any = false;
#pragma unroll
    for (int q = 0; q < ILP; ++q) {
      const uint32_t nx = rx_next<ZERO, SLOW>(rec[q].x, rec[q].y, (uint16_t)b[q]);
      if (in[q]) {
        slot[q] = nx;
        rec[q] = rx_struct_load(rsrc, nx, 0u, sb[q], 0);
      }
      in[q] = slot[q] < ni[q];   // after the step: no pass once the last lane leaves
      any |= in[q];
    }
  }
#else
  for (;;) {
    bool in[ILP];
    uint32_t b[ILP];
    bool any = false;
#pragma unroll
    for (int q = 0; q < ILP; ++q) {
      in[q] = slot[q] < ni[q];
      any |= in[q];
      // a lane at its leaf reads its own column of word 0 (conflict-free)
      b[q] = lds_u16(rx_bin_addr(rec[q].x, in[q], lane_off));
    }
#pragma unroll
    for (int q = 0; q < ILP; ++q) {
      const uint32_t nx = rx_next<ZERO, SLOW>(rec[q].x, rec[q].y, (uint16_t)b[q]);
      if (in[q]) {
        slot[q] = nx;
        rec[q] = rx_struct_load(rsrc, nx, 0u, sb[q], 0);
      }
    }
    if (__ballot(any) == 0) break;   // every lane of every tree was at a leaf
  }
#endif
}

template <typename ACC, int KMAX, bool ZERO, bool SLOW, bool VIS, int ILP>
__device__ __forceinline__ void rx_walk(const KArgs& a, ACC (&acc)[KMAX], uint32_t lane_off,
                                        int64_t row, bool live) {
  const int T = a.n_trees;
  const rx_rsrc_t rsrc = rx_make_rsrc(a.rx_recs, a.rx_slots);
  rx_cu32* rx_base = reinterpret_cast<rx_cu32*>(reinterpret_cast<uintptr_t>(a.rx_base));
  rx_cu32* rx_nint = reinterpret_cast<rx_cu32*>(reinterpret_cast<uintptr_t>(a.rx_nint));
  for (int t0 = 0; t0 < T; t0 += ILP) {
    uint32_t sb[ILP], ni[ILP];   // tree's first byte and internal-slot count (SGPRs)
    uint32_t slot[ILP];          // the lane's slot in each tree
    rx_u2_t rec[ILP];            // the record gathered last
#pragma unroll
    for (int q = 0; q < ILP; ++q) {
      const int tq = (t0 + q) < T ? (t0 + q) : (T - 1);
      sb[q] = rx_base[tq] << 3;
      ni[q] = rx_nint[tq];
      slot[q] = 0u;
      rec[q] = rx_struct_load(rsrc, 0u, 0u, sb[q], 0);   // the root (or a lone leaf)
    }
    rx_descend<ZERO, SLOW, ILP>(rsrc, sb, ni, slot, rec, lane_off);
#pragma unroll
    for (int q = 0; q < ILP; ++q)
      if (t0 + q < T)
        rx_leaves<ACC, KMAX>(a, acc, t0 + q, slot[q], ni[q], rec[q].x, rec[q].y, row, live, VIS);
  }
}

template <typename XT, typename ACC, int KMAX, bool ZERO, int ILP>
__global__ void __launch_bounds__(512) rexplicit_predict_kernel(const KArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int R = blockDim.x;
  const int tid = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * R;
  const int64_t row = row0 + tid;
  const bool live = row < a.n_rows;
  volatile int* flag = reinterpret_cast<volatile int*>(smem + (size_t)a.bin_words * R * 4);
  const bool slow = rx_stage_bins<XT, ZERO>(flag, a, row0, R, tid);
  const uint32_t lane_off = (uint32_t)tid * 4u;
  ACC acc[KMAX];
  init_acc(acc, a);
  const bool vis = a.leaf_width == 1 && a.kind != TI_OUTPUT_LEAF;
  if (slow) {
    if (vis) rx_walk<ACC, KMAX, ZERO, true, true, ILP>(a, acc, lane_off, row, live);
    else rx_walk<ACC, KMAX, ZERO, true, false, ILP>(a, acc, lane_off, row, live);
  } else {
    if (vis) rx_walk<ACC, KMAX, ZERO, false, true, ILP>(a, acc, lane_off, row, live);
    else rx_walk<ACC, KMAX, ZERO, false, false, ILP>(a, acc, lane_off, row, live);
  }
  if (!live || a.kind == TI_OUTPUT_LEAF) return;
  finish_row<ACC, KMAX>(acc, a, row);
}

// ---- staged record explicit (layout 7) -------------------------------------
// Layout 6's records, walked from LDS: the workgroup copies a stage -- a run
// of consecutive trees, the 16-byte words spanning their records -- into LDS
// (global -> registers while the previous stage is walked, then one commit
// between two barriers), and the lanes walk it ILP trees at a time in
// lockstep.  A step is one ds_read_u16 (bin) and one ds_read_b64 (record)
// per tree instead of a 64-lane gather through the vector memory pipe.  The
// LDS allocation is at least kLxMinLds (host), so the bin read of a lane at
// its leaf -- an address made of value bits -- stays inside it unclamped.
__device__ __forceinline__ rx_u2_t lx_rec(uint32_t byte_addr) {
  const uint64_t v = *reinterpret_cast<const __attribute__((address_space(3))) uint64_t*>(
      static_cast<uintptr_t>(byte_addr));
  rx_u2_t r;
  r.x = (uint32_t)v;
  r.y = (uint32_t)(v >> 32);
  return r;
}

// Layout 7 records are layout 6's with the children as byte offsets in the
// tree (slot x 8; trees of <= 8,191 slots), so a child's LDS address is one
// add to the tree's base.  The step is branch-free: a lane at its leaf keeps
// its byte offset and re-reads its leaf record, and reads its own column of
// bin word 0 (conflict-free) instead of an address made of value bits.  (Exec-
// masking the record reads instead, as layout 6 masks its gathers, measured
// 8.4 vs 6.5 ms on C3: the branches cost the compiler's counted LDS waits.)
template <typename ACC, int KMAX, bool ZERO, bool SLOW, bool VIS, int ILP>
__device__ __forceinline__ void lx_stage(const KArgs& a, ACC (&acc)[KMAX], int t0, int t1,
                                         uint32_t sbase, uint32_t lane_off, int64_t row,
                                         bool live) {
  rx_cu32* rx_base = reinterpret_cast<rx_cu32*>(reinterpret_cast<uintptr_t>(a.rx_base));
  rx_cu32* rx_nint = reinterpret_cast<rx_cu32*>(reinterpret_cast<uintptr_t>(a.rx_nint));
  for (int j = t0; j < t1; j += ILP) {
    uint32_t base[ILP], ni8[ILP], at[ILP];   // tree base (LDS), internal bytes, lane's byte
    rx_u2_t rec[ILP];
#pragma unroll
    for (int q = 0; q < ILP; ++q) {
      const int tq = (j + q) < t1 ? (j + q) : (t1 - 1);
      base[q] = sbase + (rx_base[tq] << 3);
      ni8[q] = rx_nint[tq] << 3;
      at[q] = 0u;
      rec[q] = lx_rec(base[q]);
    }
    for (;;) {
      bool in[ILP];
      uint32_t b[ILP];
      bool any = false;
#pragma unroll
      for (int q = 0; q < ILP; ++q) {
        in[q] = at[q] < ni8[q];
        any |= in[q];
        b[q] = lds_u16(rx_bin_addr(rec[q].x, in[q], lane_off));
      }
#pragma unroll
      for (int q = 0; q < ILP; ++q) {
        const uint32_t nx = rx_next<ZERO, SLOW>(rec[q].x, rec[q].y, (uint16_t)b[q]);
        at[q] = in[q] ? nx : at[q];
        rec[q] = lx_rec(base[q] + at[q]);
      }
      if (__ballot(any) == 0) break;
    }
#pragma unroll
    for (int q = 0; q < ILP; ++q)
      if (j + q < t1)
        rx_leaves<ACC, KMAX>(a, acc, j + q, at[q] >> 3, ni8[q] >> 3, rec[q].x, rec[q].y, row, live,
                             VIS);
  }
}

template <typename XT, typename ACC, int KMAX, bool ZERO, int ILP>
__global__ void __launch_bounds__(512) lexplicit_predict_kernel(const KArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int PF = 8;   // = kLxPf (host): a stage is at most PF x 16 B x R
  const int R = blockDim.x;
  const int tid = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * R;
  const int64_t row = row0 + tid;
  const bool live = row < a.n_rows;
  volatile int* flag = reinterpret_cast<volatile int*>(smem + (size_t)a.bin_words * R * 4);
  u32x4* stage = reinterpret_cast<u32x4*>(smem + a.stage_off);
  const uint32_t lane_off = (uint32_t)tid * 4u;
  rx_cu32* rx_base = reinterpret_cast<rx_cu32*>(reinterpret_cast<uintptr_t>(a.rx_base));
  rx_cu32* sst = reinterpret_cast<rx_cu32*>(reinterpret_cast<uintptr_t>(a.stage_start));
  const unsigned char* recs = reinterpret_cast<const unsigned char*>(a.rx_recs);
  const int NS = a.n_stages;
  // a stage's span: the 16-byte words from its first tree's slot 0 to the
  // end of its last tree
  auto lo_of = [&](int s) { return (rx_base[sst[s]] << 3) & ~15u; };
  auto n16_of = [&](int s) { return (int)((((rx_base[sst[s + 1]] << 3) + 15u) & ~15u) - lo_of(s)) >> 4; };
  u32x4 pf[PF];
  prefetch_n<PF>(pf, reinterpret_cast<const u32x4*>(recs + lo_of(0)), n16_of(0), tid, R);
  const bool slow = rx_stage_bins<XT, ZERO>(flag, a, row0, R, tid, stage);
  const bool vis = a.leaf_width == 1 && a.kind != TI_OUTPUT_LEAF;
  ACC acc[KMAX];
  init_acc(acc, a);
  for (int s = 0; s < NS; ++s) {
    const int t0 = (int)sst[s], t1 = (int)sst[s + 1];
    const uint32_t lo = lo_of(s);
    __syncthreads();   // the previous stage's walk is over
    commit_n<PF>(pf, stage, n16_of(s), tid, R);
    __syncthreads();
    const int sn = s + 1 < NS ? s + 1 : s;
    prefetch_n<PF>(pf, reinterpret_cast<const u32x4*>(recs + lo_of(sn)), n16_of(sn), tid, R);
    const uint32_t sbase = (uint32_t)a.stage_off - lo;   // LDS address = sbase + record byte
    if (slow) {
      if (vis) lx_stage<ACC, KMAX, ZERO, true, true, ILP>(a, acc, t0, t1, sbase, lane_off, row, live);
      else lx_stage<ACC, KMAX, ZERO, true, false, ILP>(a, acc, t0, t1, sbase, lane_off, row, live);
    } else {
      if (vis) lx_stage<ACC, KMAX, ZERO, false, true, ILP>(a, acc, t0, t1, sbase, lane_off, row, live);
      else lx_stage<ACC, KMAX, ZERO, false, false, ILP>(a, acc, t0, t1, sbase, lane_off, row, live);
    }
  }
  if (!live || a.kind == TI_OUTPUT_LEAF) return;
  finish_row<ACC, KMAX>(acc, a, row);
}

// ---- heap top + record bottom (layout 8) -----------------------------------
// Deep forests whose trees are far larger than a stage (C4: sklearn depth 16,
// ~7k nodes a tree) walk layout 6's gathers for every level, and those
// gathers bound the kernel (TD busy ~0.9).  Layout 8 stages the top D0 levels
// of each tree in LDS as a complete heap of layout 6's x words (1-based: node
// i's children are 2i and 2i+1; below a shallow leaf, padding words that
// always go left), followed at heap positions [2^D0, 2^(D0+1)) by the layout-6
// slot where the walk continues (an internal node at depth D0, or the leaf
// that ended the path above it).  A lane walks the top as the binned heap
// kernel does -- the bin read and the read of the two children together, one
// LDS round trip per level, every lane busy at every level -- and the rest of
// the tree by layout 6's exec-masked gathers from that slot.  Leaves are
// added in tree order, so sums are layout 6's, bit for bit.
template <bool ZERO, bool B8 = false>
__device__ __forceinline__ bool rx_right_slow(uint32_t x, uint32_t b) {
  using W = RxBins<B8>;
  constexpr uint32_t kNan = W::template nan_code<ZERO>();
  bool right = (x >> 16) < b;
  if (ZERO) right = right != (((b & 1u) != 0u) && ((x & W::kZeroFlip) != 0u));
  if (b == kNan) right = (x & W::kNanLeft) == 0u;
  return right;
}

template <typename ACC, int KMAX, bool ZERO, bool SLOW, bool VIS, int ILP>
__device__ __forceinline__ void hx_stage(const KArgs& a, ACC (&acc)[KMAX], const rx_rsrc_t rsrc,
                                         const unsigned char* stage, int t0, int cnt,
                                         uint32_t lane_off, int64_t row, bool live) {
  rx_cu32* rx_base = reinterpret_cast<rx_cu32*>(reinterpret_cast<uintptr_t>(a.rx_base));
  rx_cu32* rx_nint = reinterpret_cast<rx_cu32*>(reinterpret_cast<uintptr_t>(a.rx_nint));
  const int D0 = a.depth;
  const int64_t stride = a.tree_stride;
  for (int j = 0; j < cnt; j += ILP) {
    const uint32_t* tp[ILP];
    uint32_t idx[ILP], nd[ILP];
#pragma unroll
    for (int q = 0; q < ILP; ++q) {
      const int tq = (j + q) < cnt ? (j + q) : (cnt - 1);
      tp[q] = reinterpret_cast<const uint32_t*>(stage + (int64_t)tq * stride);
      idx[q] = 1u;
      nd[q] = tp[q][1];   // the root: one broadcast read
    }
    for (int l = 0; l < D0; ++l) {   // the last level selects the bottom slot
      uint32_t b[ILP];
      uint2 pr[ILP];
#pragma unroll
      for (int q = 0; q < ILP; ++q) {
        b[q] = lds_u16((nd[q] & kRxOffMask) | lane_off);
        pr[q] = *reinterpret_cast<const uint2*>(tp[q] + 2u * idx[q]);
      }
#pragma unroll
      for (int q = 0; q < ILP; ++q) {
        if (!SLOW) {
          // right = rank < bin, the child word from the pair, idx = 2 idx + right
          asm("v_cmp_lt_u32_sdwa vcc, %0, %2 src0_sel:WORD_1 src1_sel:DWORD\n\t"
              "v_cndmask_b32 %0, %3, %4, vcc\n\t"
              "v_addc_co_u32 %1, vcc, %1, %1, vcc"
              : "+v"(nd[q]), "+v"(idx[q]) : "v"(b[q]), "v"(pr[q].x), "v"(pr[q].y)
              : "vcc");
        } else {
          const bool right = rx_right_slow<ZERO>(nd[q], b[q]);
          idx[q] = idx[q] + idx[q] + (uint32_t)right;
          nd[q] = right ? pr[q].y : pr[q].x;
        }
      }
    }
    uint32_t sb[ILP], ni[ILP], slot[ILP];
    rx_u2_t rec[ILP];
#pragma unroll
    for (int q = 0; q < ILP; ++q) {
      const int tq = t0 + ((j + q) < cnt ? (j + q) : (cnt - 1));
      sb[q] = rx_base[tq] << 3;
      ni[q] = rx_nint[tq];
      slot[q] = nd[q];
    }
#pragma unroll
    for (int q = 0; q < ILP; ++q) rec[q] = rx_struct_load(rsrc, slot[q], 0u, sb[q], 0);
    rx_descend<ZERO, SLOW, ILP>(rsrc, sb, ni, slot, rec, lane_off);
#pragma unroll
    for (int q = 0; q < ILP; ++q)
      if (j + q < cnt)
        rx_leaves<ACC, KMAX>(a, acc, t0 + j + q, slot[q], ni[q], rec[q].x, rec[q].y, row, live,
                             VIS);
  }
}

// LDS: [bin image (bin_words * R u32)] [flag] ... [stage at stage_off: S tops]
template <typename XT, typename ACC, int KMAX, bool ZERO, int ILP>
__global__ void __launch_bounds__(512) hexplicit_predict_kernel(const KArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int PF = 8;   // = kHxPf (host): a stage is at most PF x 16 B x R
  const int R = blockDim.x;
  const int tid = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * R;
  const int64_t row = row0 + tid;
  const bool live = row < a.n_rows;
  volatile int* flag = reinterpret_cast<volatile int*>(smem + (size_t)a.bin_words * R * 4);
  unsigned char* stage = smem + a.stage_off;
  const uint32_t lane_off = (uint32_t)tid * 4u;
  const int T = a.n_trees;
  const int S = a.stage_trees;
  const int64_t stride = a.tree_stride;
  const rx_rsrc_t rsrc = rx_make_rsrc(a.rx_recs, a.rx_slots);
  u32x4 pf[PF];
  prefetch_n<PF>(pf, reinterpret_cast<const u32x4*>(a.trees),
                 (int)(((int64_t)(T < S ? T : S) * stride) >> 4), tid, R);
  const bool slow = rx_stage_bins<XT, ZERO, true>(flag, a, row0, R, tid, stage);
  const bool vis = a.leaf_width == 1 && a.kind != TI_OUTPUT_LEAF;
  ACC acc[KMAX];
  init_acc(acc, a);
  const int last0 = ((T - 1) / S) * S;
  for (int t0 = 0; t0 < T; t0 += S) {
    const int cnt = (T - t0) < S ? (T - t0) : S;
    __syncthreads();   // the previous stage's walk is over
    commit_n<PF>(pf, reinterpret_cast<u32x4*>(stage), (int)(((int64_t)cnt * stride) >> 4), tid, R);
    __syncthreads();
    {
      const int tn = t0 + S <= last0 ? t0 + S : last0;
      const int cn = (T - tn) < S ? (T - tn) : S;
      prefetch_n<PF>(pf, reinterpret_cast<const u32x4*>(a.trees + (int64_t)tn * stride),
                     (int)(((int64_t)cn * stride) >> 4), tid, R);
    }
    if (slow) {
      if (vis) hx_stage<ACC, KMAX, ZERO, true, true, ILP>(a, acc, rsrc, stage, t0, cnt, lane_off, row, live);
      else hx_stage<ACC, KMAX, ZERO, true, false, ILP>(a, acc, rsrc, stage, t0, cnt, lane_off, row, live);
    } else {
      if (vis) hx_stage<ACC, KMAX, ZERO, false, true, ILP>(a, acc, rsrc, stage, t0, cnt, lane_off, row, live);
      else hx_stage<ACC, KMAX, ZERO, false, false, ILP>(a, acc, rsrc, stage, t0, cnt, lane_off, row, live);
    }
  }
  if (!live || a.kind == TI_OUTPUT_LEAF) return;
  finish_row<ACC, KMAX>(acc, a, row);
}

// ---- heap top + staged bottom (layout 9) -----------------------------------
// Layout 7 with the top D0 levels of each tree as a binned heap.  Per tree the
// image holds [top: 2^(D0+1) u32 as layout 8's, except that the entries at
// [2^D0, 2^(D0+1)) are byte offsets into the bottom] [bottom: layout 7's
// records of the nodes at depth >= D0 and of every leaf, children as byte
// offsets from the bottom's start], padded to 16 bytes; stages are runs of
// consecutive trees, copied as layout 7 copies them.  A lane walks the top D0
// levels with one LDS round trip and 3 VALU a level and no lane idle (the
// lockstep of layout 7 costs two round trips and 8 VALU a step, and its
// group runs for its deepest path), then the bottom in layout 7's lockstep.
// KArgs: trees = image, depth = D0, rx_base = byte offset of each tree in the
// image [T+1], rx_nint = internal nodes of each bottom [T].
template <typename ACC, int KMAX, bool ZERO, bool SLOW, bool VIS, int ILP, bool B8>
__device__ __forceinline__ void tx_stage(const KArgs& a, ACC (&acc)[KMAX], int t0, int t1,
                                         uint32_t sbase, uint32_t lane_off, int64_t row,
                                         bool live) {
  rx_cu32* tx_off = reinterpret_cast<rx_cu32*>(reinterpret_cast<uintptr_t>(a.rx_base));
  rx_cu32* tx_nint = reinterpret_cast<rx_cu32*>(reinterpret_cast<uintptr_t>(a.rx_nint));
  const int D0 = a.depth;
  const uint32_t topb = 8u << D0;   // 2^(D0+1) u32
  for (int j = t0; j < t1; j += ILP) {
    uint32_t base[ILP], ni8[ILP], at[ILP], idx[ILP], nd[ILP];
#pragma unroll
    for (int q = 0; q < ILP; ++q) {
      const int tq = (j + q) < t1 ? (j + q) : (t1 - 1);
      base[q] = sbase + tx_off[tq];
      ni8[q] = tx_nint[tq] << 3;
      idx[q] = 1u;
      nd[q] = *reinterpret_cast<const __attribute__((address_space(3))) uint32_t*>(
          static_cast<uintptr_t>(base[q] + 4u));   // the root: one broadcast read
    }
    for (int l = 0; l < D0; ++l) {   // the last level selects the bottom entry
      uint32_t b[ILP];
      rx_u2_t pr[ILP];
#pragma unroll
      for (int q = 0; q < ILP; ++q) {
        b[q] = lds_rxbin<B8>((nd[q] & RxBins<B8>::kOffMask) | lane_off);
        pr[q] = lx_rec(base[q] + 8u * idx[q]);
      }
#pragma unroll
      for (int q = 0; q < ILP; ++q) {
        if (!SLOW) {
          asm("v_cmp_lt_u32_sdwa vcc, %0, %2 src0_sel:WORD_1 src1_sel:DWORD\n\t"
              "v_cndmask_b32 %0, %3, %4, vcc\n\t"
              "v_addc_co_u32 %1, vcc, %1, %1, vcc"
              : "+v"(nd[q]), "+v"(idx[q]) : "v"(b[q]), "v"(pr[q].x), "v"(pr[q].y)
              : "vcc");
        } else {
          const bool right = rx_right_slow<ZERO, B8>(nd[q], b[q]);
          idx[q] = idx[q] + idx[q] + (uint32_t)right;
          nd[q] = right ? pr[q].y : pr[q].x;
        }
      }
    }
    rx_u2_t rec[ILP];
#pragma unroll
    for (int q = 0; q < ILP; ++q) {
      base[q] += topb;   // the bottom
      at[q] = nd[q];
      rec[q] = lx_rec(base[q] + at[q]);
    }
    for (;;) {
      bool in[ILP];
      uint32_t b[ILP];
      bool any = false;
#pragma unroll
      for (int q = 0; q < ILP; ++q) {
        in[q] = at[q] < ni8[q];
        any |= in[q];
        b[q] = lds_rxbin<B8>(rx_bin_addr<B8>(rec[q].x, in[q], lane_off));
      }
#pragma unroll
      for (int q = 0; q < ILP; ++q) {
        const uint32_t nx = rx_next<ZERO, SLOW, B8>(rec[q].x, rec[q].y, (uint16_t)b[q]);
        at[q] = in[q] ? nx : at[q];
        rec[q] = lx_rec(base[q] + at[q]);
      }
      if (__ballot(any) == 0) break;
    }
#pragma unroll
    for (int q = 0; q < ILP; ++q)
      if (j + q < t1)
        rx_leaves<ACC, KMAX>(a, acc, j + q, at[q] >> 3, ni8[q] >> 3, rec[q].x, rec[q].y, row, live,
                             VIS);
  }
}

template <typename XT, typename ACC, int KMAX, bool ZERO, int ILP, bool B8 = false>
__global__ void __launch_bounds__(512) texplicit_predict_kernel(const KArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int PF = 8;   // = kLxPf (host): a stage is at most PF x 16 B x R
  const int R = blockDim.x;
  const int tid = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * R;
  const int64_t row = row0 + tid;
  const bool live = row < a.n_rows;
  volatile int* flag = reinterpret_cast<volatile int*>(smem + (size_t)a.bin_words * R * 4);
  u32x4* stage = reinterpret_cast<u32x4*>(smem + a.stage_off);
  const uint32_t lane_off = (uint32_t)tid * 4u;
  rx_cu32* tx_off = reinterpret_cast<rx_cu32*>(reinterpret_cast<uintptr_t>(a.rx_base));
  rx_cu32* sst = reinterpret_cast<rx_cu32*>(reinterpret_cast<uintptr_t>(a.stage_start));
  const unsigned char* img = a.trees;
  const int NS = a.n_stages;
  auto lo_of = [&](int s) { return tx_off[sst[s]]; };   // trees start 16-byte aligned
  auto n16_of = [&](int s) { return (int)((tx_off[sst[s + 1]] - tx_off[sst[s]]) >> 4); };
  u32x4 pf[PF];
  prefetch_u<PF>(pf, reinterpret_cast<const u32x4*>(img + lo_of(0)), n16_of(0), tid, R);
  const bool slow = rx_stage_bins<XT, ZERO, false, B8>(flag, a, row0, R, tid, stage);
  const bool vis = a.leaf_width == 1 && a.kind != TI_OUTPUT_LEAF;
  ACC acc[KMAX];
  init_acc(acc, a);
  for (int s = 0; s < NS; ++s) {
    const int t0 = (int)sst[s], t1 = (int)sst[s + 1];
    const uint32_t lo = lo_of(s);
    __syncthreads();   // the previous stage's walk is over
    commit_u<PF>(pf, stage, n16_of(s), tid, R);
    __syncthreads();
    const int sn = s + 1 < NS ? s + 1 : s;
    prefetch_u<PF>(pf, reinterpret_cast<const u32x4*>(img + lo_of(sn)), n16_of(sn), tid, R);
    const uint32_t sbase = (uint32_t)a.stage_off - lo;   // LDS address = sbase + image byte
    if (slow) {
      if (vis) tx_stage<ACC, KMAX, ZERO, true, true, ILP, B8>(a, acc, t0, t1, sbase, lane_off, row, live);
      else tx_stage<ACC, KMAX, ZERO, true, false, ILP, B8>(a, acc, t0, t1, sbase, lane_off, row, live);
    } else {
      if (vis) tx_stage<ACC, KMAX, ZERO, false, true, ILP, B8>(a, acc, t0, t1, sbase, lane_off, row, live);
      else tx_stage<ACC, KMAX, ZERO, false, false, ILP, B8>(a, acc, t0, t1, sbase, lane_off, row, live);
    }
  }
  if (!live || a.kind == TI_OUTPUT_LEAF) return;
  finish_row<ACC, KMAX>(acc, a, row);
}


// ---- layout 9 with the compact u8 bottom (plan_tx8) ------------------------
// Top as layout 9's (the rank is byte 2 of an x word here, so the compare
// selects BYTE_2; byte 3 holds the pair index); then per bottom step one LDS
// round trip: the u8 bin of the lane's node and the 8-byte pair of its
// children (position 2k', k' = byte 3) at once, one compare and one select,
// no lane mask: a leaf's word loops on itself (rank 0xFF at even positions,
// 0 at odd ones).  The group's loop ends when every lane of every tree holds
// a leaf word (kLeaf in all of them).  A leaf's position 2k' + (rank == 0)
// indexes the forest's position tables: the value (VIS) is loaded when the
// group ends and added when the next group ends (tree order kept, the load's
// latency hidden behind a walk); ordinals (leaf ids, vector leaves) at once.
template <bool ZERO>
__device__ __forceinline__ bool t8_right_slow(uint32_t x, uint32_t b) {
  using W = RxBins<true>;
  bool right = ((x >> 16) & 0xFFu) < b;
  if (ZERO) right = right != (((b & 1u) != 0u) && ((x & W::kZeroFlip) != 0u));
  if (b == 0u) right = (x & W::kNanLeft) == 0u;
  return right;
}

template <typename ACC, int KMAX, int ILP>
__device__ __forceinline__ void t8_flush(const KArgs& a, ACC (&acc)[KMAX], const ACC (&pend)[ILP],
                                         const int (&pend_t)[ILP]) {
#pragma unroll
  for (int q = 0; q < ILP; ++q)
    if (pend_t[q] >= 0) add_leaf<ACC, KMAX>(acc, &pend[q], 0, 1, a.tree_group[pend_t[q]]);
}

template <typename ACC, int KMAX, bool ZERO, bool SLOW, bool VIS, int ILP>
__device__ __forceinline__ void t8_stage(const KArgs& a, ACC (&acc)[KMAX], int t0, int t1,
                                         uint32_t sbase, uint32_t lane_off, int64_t row, bool live,
                                         ACC (&pend)[ILP], int (&pend_t)[ILP]) {
  using W = RxBins<true>;
  rx_cu32* tx_off = reinterpret_cast<rx_cu32*>(reinterpret_cast<uintptr_t>(a.rx_base));
  rx_cu32* tx_pos = reinterpret_cast<rx_cu32*>(reinterpret_cast<uintptr_t>(a.tx_pos));
  const int D0 = a.depth;
  const uint32_t topb = 8u << D0;   // 2^(D0+1) u32
  for (int j = t0; j < t1; j += ILP) {
    uint32_t base[ILP], idx[ILP], nd[ILP];
#pragma unroll
    for (int q = 0; q < ILP; ++q) {
      const int tq = (j + q) < t1 ? (j + q) : (t1 - 1);
      base[q] = sbase + tx_off[tq];
      idx[q] = 1u;
      nd[q] = *reinterpret_cast<const __attribute__((address_space(3))) uint32_t*>(
          static_cast<uintptr_t>(base[q] + 4u));   // the root: one broadcast read
    }
    for (int l = 0; l < D0; ++l) {   // the last level selects the bottom entry
      uint32_t b[ILP];
      rx_u2_t pr[ILP];
#pragma unroll
      for (int q = 0; q < ILP; ++q) {
        b[q] = lds_u8((nd[q] & W::kNodeMask) | lane_off);
        pr[q] = lx_rec(base[q] + 8u * idx[q]);
      }
#pragma unroll
      for (int q = 0; q < ILP; ++q) {
        if (!SLOW) {
          asm("v_cmp_lt_u32_sdwa vcc, %0, %2 src0_sel:BYTE_2 src1_sel:DWORD\n\t"
              "v_cndmask_b32 %0, %3, %4, vcc\n\t"
              "v_addc_co_u32 %1, vcc, %1, %1, vcc"
              : "+v"(nd[q]), "+v"(idx[q]) : "v"(b[q]), "v"(pr[q].x), "v"(pr[q].y)
              : "vcc");
        } else {
          const bool right = t8_right_slow<ZERO>(nd[q], b[q]);
          idx[q] = idx[q] + idx[q] + (uint32_t)right;
          nd[q] = right ? pr[q].y : pr[q].x;
        }
      }
    }
    uint32_t x[ILP];
#pragma unroll
    for (int q = 0; q < ILP; ++q) {
      base[q] += topb;   // the bottom: u32 words by position
      x[q] = *reinterpret_cast<const __attribute__((address_space(3))) uint32_t*>(
          static_cast<uintptr_t>(base[q] + 4u * nd[q]));
    }
    for (;;) {
      uint32_t all = x[0];
#pragma unroll
      for (int q = 1; q < ILP; ++q) all &= x[q];
      if (__ballot((all & W::kLeaf) == 0u) == 0) break;   // every lane of every tree at a leaf
      uint32_t b[ILP];
      rx_u2_t pr[ILP];
#pragma unroll
      for (int q = 0; q < ILP; ++q) {
        b[q] = lds_u8((x[q] & W::kNodeMask) | lane_off);
        pr[q] = lx_rec(base[q] + ((x[q] >> 24) << 3));
      }
#pragma unroll
      for (int q = 0; q < ILP; ++q) {
        if (!SLOW) {
          asm("v_cmp_lt_u32_sdwa vcc, %0, %1 src0_sel:BYTE_2 src1_sel:DWORD\n\t"
              "v_cndmask_b32 %0, %2, %3, vcc"
              : "+v"(x[q]) : "v"(b[q]), "v"(pr[q].x), "v"(pr[q].y) : "vcc");
        } else {
          x[q] = t8_right_slow<ZERO>(x[q], b[q]) ? pr[q].y : pr[q].x;
        }
      }
    }
    uint32_t li[ILP];   // the leaf's index in the position tables
#pragma unroll
    for (int q = 0; q < ILP; ++q) {
      const int tq = (j + q) < t1 ? (j + q) : (t1 - 1);
      li[q] = tx_pos[tq] + ((x[q] >> 23) & ~1u) + (((x[q] >> 16) & 0xFFu) == 0u ? 1u : 0u);
    }
    if (VIS) {
      t8_flush<ACC, KMAX, ILP>(a, acc, pend, pend_t);   // the previous group's leaves
#pragma unroll
      for (int q = 0; q < ILP; ++q) {
        pend[q] = static_cast<const ACC*>(a.tx_vals)[li[q]];
        pend_t[q] = (j + q) < t1 ? (j + q) : -1;
      }
    } else {
#pragma unroll
      for (int q = 0; q < ILP; ++q) {
        const int t = j + q;
        if (t < t1) {
          const int64_t lf = a.leaf_base[t] + (int64_t)a.tx_ord[li[q]];
          if (a.kind == TI_OUTPUT_LEAF) {
            if (live) static_cast<int32_t*>(a.out)[row * a.n_trees + t] = a.exp_leaf_ids[lf];
          } else {
            add_leaf<ACC, KMAX>(acc, static_cast<const ACC*>(a.leaves) + lf * a.leaf_width, 0,
                                a.leaf_width, a.tree_group[t]);
          }
        }
      }
    }
  }
}

template <typename XT, typename ACC, int KMAX, bool ZERO, int ILP>
__global__ void __launch_bounds__(512) t8explicit_predict_kernel(const KArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int PF = 8;   // = kLxPf (host): a stage is at most PF x 16 B x R
  const int R = blockDim.x;
  const int tid = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * R;
  const int64_t row = row0 + tid;
  const bool live = row < a.n_rows;
  volatile int* flag = reinterpret_cast<volatile int*>(smem + (size_t)a.bin_words * R * 4);
  u32x4* stage = reinterpret_cast<u32x4*>(smem + a.stage_off);
  const uint32_t lane_off = (uint32_t)tid * 4u;
  rx_cu32* tx_off = reinterpret_cast<rx_cu32*>(reinterpret_cast<uintptr_t>(a.rx_base));
  rx_cu32* sst = reinterpret_cast<rx_cu32*>(reinterpret_cast<uintptr_t>(a.stage_start));
  const unsigned char* img = a.trees;
  const int NS = a.n_stages;
  auto lo_of = [&](int s) { return tx_off[sst[s]]; };   // trees start 16-byte aligned
  auto n16_of = [&](int s) { return (int)((tx_off[sst[s + 1]] - tx_off[sst[s]]) >> 4); };
  u32x4 pf[PF];
  prefetch_u<PF>(pf, reinterpret_cast<const u32x4*>(img + lo_of(0)), n16_of(0), tid, R);
  const bool slow = rx_stage_bins<XT, ZERO, false, true>(flag, a, row0, R, tid, stage);
  const bool vis = a.leaf_width == 1 && a.kind != TI_OUTPUT_LEAF;
  ACC acc[KMAX];
  init_acc(acc, a);
  ACC pend[ILP];   // the previous group's leaf values (t8_stage)
  int pend_t[ILP];
#pragma unroll
  for (int q = 0; q < ILP; ++q) {
    pend[q] = ACC(0);
    pend_t[q] = -1;
  }
  for (int s = 0; s < NS; ++s) {
    const int t0 = (int)sst[s], t1 = (int)sst[s + 1];
    const uint32_t lo = lo_of(s);
    __syncthreads();   // the previous stage's walk is over
    commit_u<PF>(pf, stage, n16_of(s), tid, R);
    __syncthreads();
    const int sn = s + 1 < NS ? s + 1 : s;
    prefetch_u<PF>(pf, reinterpret_cast<const u32x4*>(img + lo_of(sn)), n16_of(sn), tid, R);
    const uint32_t sbase = (uint32_t)a.stage_off - lo;   // LDS address = sbase + image byte
    if (slow) {
      if (vis) t8_stage<ACC, KMAX, ZERO, true, true, ILP>(a, acc, t0, t1, sbase, lane_off, row, live, pend, pend_t);
      else t8_stage<ACC, KMAX, ZERO, true, false, ILP>(a, acc, t0, t1, sbase, lane_off, row, live, pend, pend_t);
    } else {
      if (vis) t8_stage<ACC, KMAX, ZERO, false, true, ILP>(a, acc, t0, t1, sbase, lane_off, row, live, pend, pend_t);
      else t8_stage<ACC, KMAX, ZERO, false, false, ILP>(a, acc, t0, t1, sbase, lane_off, row, live, pend, pend_t);
    }
  }
  if (vis) t8_flush<ACC, KMAX, ILP>(a, acc, pend, pend_t);
  if (!live || a.kind == TI_OUTPUT_LEAF) return;
  finish_row<ACC, KMAX>(acc, a, row);
}

// ---- layout 9 with the compact u16 bottom (plan_tx16) -----------------------
// The u8 compact bottom's step for u16 bins (C3: ~2,500 thresholds a feature).
// A bottom node is one u32: rank in the high half (the compare reads WORD_1,
// as the record walk's), the bin's byte offset in the low half with the lane
// part cleared (bit 0 NaN-left, bit 1 the half-word, the word index above the
// lane bits), and the children's pair index k' in bits 2-9 -- inside the lane
// part, which the bin address masks off (a.bin_mask).  Children sit side by
// side at positions 2k', 2k'+1, so a step is one LDS round trip (the u16 bin
// and the 8-byte pair) and 5 VALU, against the record bottom's two round trips
// and 7 VALU.  A leaf loops on itself (rank 0xFFFF at even positions: never
// right, NaN-left; rank 0 at odd ones: always right, since every real bin is
// >= 1 and a NaN takes the NaN-left bit) with bin offset 0, so a finished
// lane reads its own column of word 0 (conflict-free, a real bin: a read of
// anything else could return 0 and send an odd leaf to its sibling).  No
// internal node has rank 0 or 0xFFFF (plan_tx16 checks), so the group's loop
// ends when every tree's rank is one of those: (x + 0x10000) < 0x20000.  LightGBM's
// zero flip has no bit left in the word: zero-missing forests keep one flag
// bit per position in a 64-byte table between the top and the bottom, read by
// the slow step (tiles holding an exact 0 or a NaN), which tracks the node's
// position.  Leaf values come from the position tables as in t8_stage.
constexpr uint32_t kT16ZfBytes = 64;   // zero-flip bits of <= 512 positions

template <bool ZERO>
__device__ __forceinline__ bool t16_right_slow(uint32_t x, uint32_t b, bool zf) {
  constexpr uint32_t kNan = RxBins<false>::template nan_code<ZERO>();
  bool right = (x >> 16) < b;
  if (ZERO) right = right != (((b & 1u) != 0u) && zf);
  if (b == kNan) right = (x & 1u) == 0u;
  return right;
}

// The two-lanes-a-row walk (t16split_predict_kernel): a lane's partner
// (lane l + 32 for l < 32) holds the same row and walks the other half of
// each group of 2 x ILP trees.  v_permlane32_swap hands the lower half the
// upper half's values (ISA: vdst lanes 32-63 <-> vsrc lanes 0-31; the
// builtin returns {vdst, vsrc}, so lane l < 32 finds lane l + 32's value in
// the second); the upper half gets its own back and its sums are never used.
__device__ __forceinline__ uint32_t from_upper_half(uint32_t v) {
  return __builtin_amdgcn_permlane32_swap(v, v, false, false)[1];
}
template <typename ACC>
__device__ __forceinline__ ACC from_upper_half(ACC v) {
  if constexpr (sizeof(ACC) == 8) {
    const double d = static_cast<double>(v);
    const uint32_t lo = from_upper_half((uint32_t)__double2loint(d));
    const uint32_t hi = from_upper_half((uint32_t)__double2hiint(d));
    return static_cast<ACC>(__hiloint2double((int)hi, (int)lo));
  } else {
    return static_cast<ACC>(__uint_as_float(from_upper_half(__float_as_uint(static_cast<float>(v)))));
  }
}

// A split group's leaves in the library's order: the lower lane's own trees
// j .. j + ILP - 1, then its partner's j + ILP .. j + 2 ILP - 1.  The swaps
// run on all 64 lanes before any lane branches.
template <typename ACC, int KMAX, int ILP>
__device__ __forceinline__ void t16_flush_split(const KArgs& a, ACC (&acc)[KMAX],
                                                const ACC (&pend)[ILP], const int (&pend_t)[ILP]) {
  ACC pp[ILP];
  int pt[ILP];
#pragma unroll
  for (int q = 0; q < ILP; ++q) {
    pp[q] = from_upper_half<ACC>(pend[q]);
    pt[q] = (int)from_upper_half((uint32_t)pend_t[q]);
  }
  t8_flush<ACC, KMAX, ILP>(a, acc, pend, pend_t);
  t8_flush<ACC, KMAX, ILP>(a, acc, pp, pt);
}

template <typename ACC, int KMAX, bool ZERO, bool SLOW, bool VIS, int ILP, bool SPLIT = false>
__device__ __forceinline__ void t16_stage(const KArgs& a, ACC (&acc)[KMAX], int t0, int t1,
                                          uint32_t sbase, uint32_t lane_off, int64_t row,
                                          bool live, ACC (&pend)[ILP], int (&pend_t)[ILP],
                                          int half = 0) {
  rx_cu32* tx_off = reinterpret_cast<rx_cu32*>(reinterpret_cast<uintptr_t>(a.rx_base));
  rx_cu32* tx_pos = reinterpret_cast<rx_cu32*>(reinterpret_cast<uintptr_t>(a.tx_pos));
  const int D0 = a.depth;
  const uint32_t topb = 8u << D0;                   // 2^(D0+1) u32
  const uint32_t zfb = ZERO ? kT16ZfBytes : 0u;     // zero-flip bits before the bottom
  const uint32_t bmask = a.bin_mask;                // word index | half (the lane part cleared)
  for (int jg = t0; jg < t1; jg += (SPLIT ? 2 : 1) * ILP) {
    const int j = SPLIT ? jg + half * ILP : jg;   // this lane's first tree of the group
    uint32_t base[ILP], idx[ILP], nd[ILP], pos0[ILP];
#pragma unroll
    for (int q = 0; q < ILP; ++q) {
      // both halves' tree tables by wave-uniform indices (scalar loads), then
      // the lane's half selected: a lane-dependent index would make every
      // table read a vector gather
      const int ta = (jg + q) < t1 ? (jg + q) : (t1 - 1);
      const int tb = SPLIT ? ((jg + ILP + q) < t1 ? (jg + ILP + q) : (t1 - 1)) : ta;
      const uint32_t oa = tx_off[ta], ob = tx_off[tb];
      base[q] = sbase + (SPLIT && half ? ob : oa);
      if constexpr (SPLIT) {   // both loaded (scalar), then selected: a select of two
        const uint32_t pa = tx_pos[ta], pb = tx_pos[tb];   // loads became one gather
        pos0[q] = half ? pb : pa;
      }
      idx[q] = 1u;
      nd[q] = *reinterpret_cast<const __attribute__((address_space(3))) uint32_t*>(
          static_cast<uintptr_t>(base[q] + 4u));   // the root: one broadcast read per half
    }
    for (int l = 0; l < D0; ++l) {   // the top, as layout 9's (record x words)
      uint32_t b[ILP];
      rx_u2_t pr[ILP];
#pragma unroll
      for (int q = 0; q < ILP; ++q) {
        b[q] = lds_u16((nd[q] & kRxOffMask) | lane_off);
        pr[q] = lx_rec(base[q] + 8u * idx[q]);
      }
#pragma unroll
      for (int q = 0; q < ILP; ++q) {
        if (!SLOW) {
          asm("v_cmp_lt_u32_sdwa vcc, %0, %2 src0_sel:WORD_1 src1_sel:DWORD\n\t"
              "v_cndmask_b32 %0, %3, %4, vcc\n\t"
              "v_addc_co_u32 %1, vcc, %1, %1, vcc"
              : "+v"(nd[q]), "+v"(idx[q]) : "v"(b[q]), "v"(pr[q].x), "v"(pr[q].y)
              : "vcc");
        } else {
          const bool right = rx_right_slow<ZERO, false>(nd[q], b[q]);
          idx[q] = idx[q] + idx[q] + (uint32_t)right;
          nd[q] = right ? pr[q].y : pr[q].x;
        }
      }
    }
    uint32_t x[ILP], p[ILP];   // node word; its position (slow zero-missing steps only)
#pragma unroll
    for (int q = 0; q < ILP; ++q) {
      p[q] = nd[q];
      base[q] += topb + zfb;   // the bottom: u32 words by position
      x[q] = *reinterpret_cast<const __attribute__((address_space(3))) uint32_t*>(
          static_cast<uintptr_t>(base[q] + 4u * nd[q]));
    }
    for (;;) {
      // a leaf's rank is 0xFFFF or 0: x + 0x10000 < 0x20000
      uint32_t anyw = 0u;
#pragma unroll
      for (int q = 0; q < ILP; ++q) anyw |= x[q] + 0x10000u;
      if (__ballot((anyw & 0xFFFE0000u) != 0u) == 0) break;   // every lane of every tree at a leaf
      uint32_t b[ILP];
      rx_u2_t pr[ILP];
      uint32_t zb[ILP];
#pragma unroll
      for (int q = 0; q < ILP; ++q) {
        b[q] = lds_u16((x[q] & bmask) | lane_off);
        pr[q] = lx_rec(base[q] + ((x[q] & 0x3FCu) << 1));
        if (SLOW && ZERO) zb[q] = lds_u8(base[q] - zfb + (p[q] >> 3));
      }
#pragma unroll
      for (int q = 0; q < ILP; ++q) {
        if (!SLOW) {
          asm("v_cmp_lt_u32_sdwa vcc, %0, %1 src0_sel:WORD_1 src1_sel:WORD_0\n\t"
              "v_cndmask_b32 %0, %2, %3, vcc"
              : "+v"(x[q]) : "v"(b[q]), "v"(pr[q].x), "v"(pr[q].y) : "vcc");
        } else {
          const bool zf = ZERO && ((zb[q] >> (p[q] & 7u)) & 1u) != 0u;
          const bool right = t16_right_slow<ZERO>(x[q], b[q] & 0xFFFFu, zf);
          if (ZERO) p[q] = ((x[q] >> 1) & 0x1FEu) + (right ? 1u : 0u);
          x[q] = right ? pr[q].y : pr[q].x;
        }
      }
    }
    uint32_t li[ILP];   // the leaf's index in the position tables
#pragma unroll
    for (int q = 0; q < ILP; ++q) {
      const int tq = (j + q) < t1 ? (j + q) : (t1 - 1);
      li[q] = (SPLIT ? pos0[q] : tx_pos[tq]) + ((x[q] >> 1) & 0x1FEu) +
              ((x[q] >> 16) == 0u ? 1u : 0u);
    }
    if (VIS) {
      // the previous group's leaves
      if (SPLIT) t16_flush_split<ACC, KMAX, ILP>(a, acc, pend, pend_t);
      else t8_flush<ACC, KMAX, ILP>(a, acc, pend, pend_t);
#pragma unroll
      for (int q = 0; q < ILP; ++q) {
        pend[q] = static_cast<const ACC*>(a.tx_vals)[li[q]];
        pend_t[q] = (j + q) < t1 ? (j + q) : -1;
      }
    } else {
#pragma unroll
      for (int q = 0; q < ILP; ++q) {
        const int t = j + q;
        if (t < t1) {
          const int64_t lf = a.leaf_base[t] + (int64_t)a.tx_ord[li[q]];
          if (a.kind == TI_OUTPUT_LEAF) {
            if (live) static_cast<int32_t*>(a.out)[row * a.n_trees + t] = a.exp_leaf_ids[lf];
          } else if (!SPLIT) {   // (the host gives the split walk scalar leaves only)
            add_leaf<ACC, KMAX>(acc, static_cast<const ACC*>(a.leaves) + lf * a.leaf_width, 0,
                                a.leaf_width, a.tree_group[t]);
          }
        }
      }
    }
  }
}

template <typename XT, typename ACC, int KMAX, bool ZERO, int ILP>
__global__ void __launch_bounds__(512) t16explicit_predict_kernel(const KArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int PF = 8;   // = kLxPf (host): a stage is at most PF x 16 B x R
  const int R = blockDim.x;
  const int tid = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * R;
  const int64_t row = row0 + tid;
  const bool live = row < a.n_rows;
  volatile int* flag = reinterpret_cast<volatile int*>(smem + (size_t)a.bin_words * R * 4);
  u32x4* stage = reinterpret_cast<u32x4*>(smem + a.stage_off);
  const uint32_t lane_off = (uint32_t)tid * 4u;
  rx_cu32* tx_off = reinterpret_cast<rx_cu32*>(reinterpret_cast<uintptr_t>(a.rx_base));
  rx_cu32* sst = reinterpret_cast<rx_cu32*>(reinterpret_cast<uintptr_t>(a.stage_start));
  const unsigned char* img = a.trees;
  const int NS = a.n_stages;
  auto lo_of = [&](int s) { return tx_off[sst[s]]; };   // trees start 16-byte aligned
  auto n16_of = [&](int s) { return (int)((tx_off[sst[s + 1]] - tx_off[sst[s]]) >> 4); };
  u32x4 pf[PF];
  prefetch_u<PF>(pf, reinterpret_cast<const u32x4*>(img + lo_of(0)), n16_of(0), tid, R);
  const bool slow = rx_stage_bins<XT, ZERO, false, false>(flag, a, row0, R, tid, stage);
  const bool vis = a.leaf_width == 1 && a.kind != TI_OUTPUT_LEAF;
  ACC acc[KMAX];
  init_acc(acc, a);
  ACC pend[ILP];   // the previous group's leaf values
  int pend_t[ILP];
#pragma unroll
  for (int q = 0; q < ILP; ++q) {
    pend[q] = ACC(0);
    pend_t[q] = -1;
  }
  for (int s = 0; s < NS; ++s) {
    const int t0 = (int)sst[s], t1 = (int)sst[s + 1];
    const uint32_t lo = lo_of(s);
    __syncthreads();   // the previous stage's walk is over
    commit_u<PF>(pf, stage, n16_of(s), tid, R);
    __syncthreads();
    const int sn = s + 1 < NS ? s + 1 : s;
    prefetch_u<PF>(pf, reinterpret_cast<const u32x4*>(img + lo_of(sn)), n16_of(sn), tid, R);
    const uint32_t sbase = (uint32_t)a.stage_off - lo;   // LDS address = sbase + image byte
    if (slow) {
      if (vis) t16_stage<ACC, KMAX, ZERO, true, true, ILP>(a, acc, t0, t1, sbase, lane_off, row, live, pend, pend_t);
      else t16_stage<ACC, KMAX, ZERO, true, false, ILP>(a, acc, t0, t1, sbase, lane_off, row, live, pend, pend_t);
    } else {
      if (vis) t16_stage<ACC, KMAX, ZERO, false, true, ILP>(a, acc, t0, t1, sbase, lane_off, row, live, pend, pend_t);
      else t16_stage<ACC, KMAX, ZERO, false, false, ILP>(a, acc, t0, t1, sbase, lane_off, row, live, pend, pend_t);
    }
  }
  if (vis) t8_flush<ACC, KMAX, ILP>(a, acc, pend, pend_t);
  if (!live || a.kind == TI_OUTPUT_LEAF) return;
  finish_row<ACC, KMAX>(acc, a, row);
}

// Two lanes a row (round 6): the R-row tile of the u16 compact
// walk on 2R threads.  Wave w holds rows 32w .. 32w + 31 twice: lanes 0-31
// walk the first ILP trees of every group of 2 ILP, lanes 32-63 the other
// ILP, so a CU keeps twice the waves resident with the same LDS (bins,
// stage); each 32-lane half is one LDS lane group and reads 32 distinct
// rows' bins, conflict-free as the one-lane walk.  The lower lane adds the
// group's leaves in tree order (t16_flush_split) and writes the row.
template <typename XT, typename ACC, int KMAX, bool ZERO, int ILP>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) t16split_predict_kernel(const KArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int PF = 4;   // 2R threads prefetch a stage of at most kLxPf x 16 B x R
  const int NT = blockDim.x;
  const int R = NT >> 1;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int half = lane >> 5;
  const int rloc = ((tid >> 6) << 5) | (lane & 31);   // the tile row of this lane pair
  const int64_t row0 = (int64_t)blockIdx.x * R;
  const int64_t row = row0 + rloc;
  const bool live = row < a.n_rows;
  volatile int* flag = reinterpret_cast<volatile int*>(smem + (size_t)a.bin_words * R * 4);
  u32x4* stage = reinterpret_cast<u32x4*>(smem + a.stage_off);
  const uint32_t lane_off = (uint32_t)rloc * 4u;
  rx_cu32* tx_off = reinterpret_cast<rx_cu32*>(reinterpret_cast<uintptr_t>(a.rx_base));
  rx_cu32* sst = reinterpret_cast<rx_cu32*>(reinterpret_cast<uintptr_t>(a.stage_start));
  const unsigned char* img = a.trees;
  const int NS = a.n_stages;
  auto lo_of = [&](int s) { return tx_off[sst[s]]; };   // trees start 16-byte aligned
  auto n16_of = [&](int s) { return (int)((tx_off[sst[s + 1]] - tx_off[sst[s]]) >> 4); };
  // the first stage is fetched after the binning, not during it: the float64
  // binning's 5-ary search keeps 8 x 4 doubles in flight, and prefetch
  // registers live across it took the kernel past the 128 VGPRs 4 waves a
  // SIMD allow (138: 3 waves, one workgroup a CU); the exposed fetch is one
  // per tile, ~0.3 % of it
  const bool slow = rx_stage_bins<XT, ZERO, false, false>(flag, a, row0, R, tid, stage, NT);
  u32x4 pf[PF];
  prefetch_u<PF>(pf, reinterpret_cast<const u32x4*>(img + lo_of(0)), n16_of(0), tid, NT);
  const bool vis = a.leaf_width == 1 && a.kind != TI_OUTPUT_LEAF;
  ACC acc[KMAX];
  init_acc(acc, a);
  ACC pend[ILP];   // the previous group's leaf values (this lane's half)
  int pend_t[ILP];
#pragma unroll
  for (int q = 0; q < ILP; ++q) {
    pend[q] = ACC(0);
    pend_t[q] = -1;
  }
  for (int s = 0; s < NS; ++s) {
    const int t0 = (int)sst[s], t1 = (int)sst[s + 1];
    const uint32_t lo = lo_of(s);
    __syncthreads();   // the previous stage's walk is over
    commit_u<PF>(pf, stage, n16_of(s), tid, NT);
    __syncthreads();
    const int sn = s + 1 < NS ? s + 1 : s;
    prefetch_u<PF>(pf, reinterpret_cast<const u32x4*>(img + lo_of(sn)), n16_of(sn), tid, NT);
    const uint32_t sbase = (uint32_t)a.stage_off - lo;   // LDS address = sbase + image byte
    if (slow) {
      if (vis) t16_stage<ACC, KMAX, ZERO, true, true, ILP, true>(a, acc, t0, t1, sbase, lane_off, row, live, pend, pend_t, half);
      else t16_stage<ACC, KMAX, ZERO, true, false, ILP, true>(a, acc, t0, t1, sbase, lane_off, row, live, pend, pend_t, half);
    } else {
      if (vis) t16_stage<ACC, KMAX, ZERO, false, true, ILP, true>(a, acc, t0, t1, sbase, lane_off, row, live, pend, pend_t, half);
      else t16_stage<ACC, KMAX, ZERO, false, false, ILP, true>(a, acc, t0, t1, sbase, lane_off, row, live, pend, pend_t, half);
    }
  }
  if (vis) t16_flush_split<ACC, KMAX, ILP>(a, acc, pend, pend_t);
  if (!live || a.kind == TI_OUTPUT_LEAF || half) return;
  finish_row<ACC, KMAX>(acc, a, row);
}

}  // namespace ti
