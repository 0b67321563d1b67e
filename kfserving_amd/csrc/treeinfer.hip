// treeinfer.hip — libtreeinfer.so: C ABI (include/treeinfer.h) over the
// gfx950 kernels in treeinfer_kernels.h.
//
// Host responsibilities:
//   * validate the canonical SoA forest handed over by the Python loaders
//     (kfserving_amd/formats/*), which replaces the library handles built in
//     xgbserver/model.py:38-39, lgbserver/model.py:39-40,
//     sklearnserver/model.py:38;
//   * choose a device layout (heap = complete trees staged in LDS, or
//     explicit nodes) and upload one replica per device;
//   * ti_predict: shard rows in contiguous blocks over the devices (one host
//     thread per device, one stream each), H2D -> one fused kernel -> D2H.
//     This replaces XGBoosterPredict / LGBM_BoosterPredictForMat /
//     Forest*.predict at xgbserver/model.py:46-47, lgbserver/model.py:51,
//     sklearnserver/model.py:50.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <limits>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <utility>
#include <type_traits>
#include <vector>

#include "treeinfer.h"
#include "treeinfer_kernels.h"
#include "treeinfer_dispatch.h"

using ti::ExpNode;
using ti::HeapNode;
using ti::KArgs;

// ---------------------------------------------------------- TreeSHAP paths
// Every root-to-leaf path of every tree, with the splits on one feature
// merged into one element (the unique path xgboost's TreeShap keeps: a
// feature seen again is unwound and re-extended at the end, so elements are
// in order of last occurrence).  An element holds the product of the
// child/parent cover ratios of its splits (zero fraction) and the condition
// a row must meet to follow all of them (one fraction 1, else 0).
struct ShapPath {
  int32_t group;    // output group (leaf_width 1)
  int32_t n;        // elements (excluding the root's dummy element)
  int64_t first;    // first element
  int64_t leaf;     // row of the path's leaf in the leaf-value table
};
constexpr uint32_t kShapNanOk = 1u;    // NaN follows every split of the element
constexpr uint32_t kShapZeroOk = 2u;   // exact 0 follows every split (LightGBM zero rule)
constexpr uint32_t kShapEmpty = 4u;    // no non-NaN value follows (a left turn at a NaN threshold)
struct ShapElem {
  int32_t feature;
  uint32_t flags;
  double lo;        // follows iff lo < x <= hi (non-NaN, non-zero x)
  double hi;
  double zf;        // zero fraction
};

// One row per lane (64-row blocks).  Per path: the one fractions of the
// row, then the path weights extended from scratch (ExtendPath) and, per
// element, the unwound sum (UnwoundPathSum) times (one - zero) times the
// leaf value, added to the element's feature.  Path weights and one
// fractions live in LDS as [index][lane].  acc is float64 [rows, K*(F+1)];
// the last pass divides by average_divisor, writes the bias and converts to
// ACC.
template <typename XT, typename ACC>
__global__ void __launch_bounds__(64) contrib_kernel(
    const XT* __restrict__ X, int64_t rows, int64_t stride, int32_t cols, int32_t zero_map_on,
    const ShapPath* __restrict__ paths, int64_t n_paths, const ShapElem* __restrict__ elems,
    const double* __restrict__ leafv, int32_t LW, int32_t K, int32_t F, int32_t maxl,
    const double* __restrict__ bias, double divisor, double* __restrict__ acc,
    ACC* __restrict__ out) {
  extern __shared__ double shap_lds[];
  const int lane = threadIdx.x;
  const int64_t row = (int64_t)blockIdx.x * 64 + lane;
  const bool live = row < rows;
  double* w = shap_lds;                         // [maxl + 1][64]
  double* ob = shap_lds + (size_t)(maxl + 1) * 64;   // [maxl][64]
  const XT* xr = X + (live ? row : rows - 1) * stride;
  const int W = K * (F + 1);
  double* ph = acc + (live ? row : 0) * W;
  for (int64_t p = 0; p < n_paths; ++p) {
    const ShapPath P = paths[p];
    const int n = P.n;
    for (int i = 0; i < n; ++i) {
      const ShapElem e = elems[P.first + i];
      double x = e.feature < cols ? (double)xr[e.feature] : __builtin_nan("");
      if (zero_map_on && __builtin_fabs(x) <= (double)1e-35f) x = 0.0;
      bool follow;
      if (x != x) follow = (e.flags & kShapNanOk) != 0;
      else if (x == 0.0) follow = (e.flags & kShapZeroOk) != 0;
      else follow = !(e.flags & kShapEmpty) && e.lo < x && x <= e.hi;
      ob[i * 64 + lane] = follow ? 1.0 : 0.0;
    }
    w[lane] = 1.0;
    for (int d = 1; d <= n; ++d) {
      const double zf = elems[P.first + d - 1].zf;
      const double of = ob[(d - 1) * 64 + lane];
      w[d * 64 + lane] = 0.0;
      for (int i = d - 1; i >= 0; --i) {
        w[(i + 1) * 64 + lane] += of * w[i * 64 + lane] * (i + 1) / (double)(d + 1);
        w[i * 64 + lane] = zf * w[i * 64 + lane] * (d - i) / (double)(d + 1);
      }
    }
    for (int e_i = 1; e_i <= n; ++e_i) {
      const ShapElem e = elems[P.first + e_i - 1];
      const double of = ob[(e_i - 1) * 64 + lane];
      const double zf = e.zf;
      double next = w[n * 64 + lane];
      double total = 0.0;
      for (int i = n - 1; i >= 0; --i) {
        if (of != 0.0) {
          const double tmp = next * (n + 1) / ((i + 1) * of);
          total += tmp;
          next = w[i * 64 + lane] - tmp * zf * (n - i) / (double)(n + 1);
        } else {
          total += (w[i * 64 + lane] / zf) / ((n - i) / (double)(n + 1));
        }
      }
      const double scale = total * (of - zf);
      if (live) {
        if (LW == 1) {
          ph[P.group * (F + 1) + e.feature] += scale * leafv[P.leaf];
        } else {
          for (int k = 0; k < LW; ++k) ph[k * (F + 1) + e.feature] += scale * leafv[P.leaf * LW + k];
        }
      }
    }
  }
  if (!live) return;
  ACC* o = out + row * W;
  for (int g = 0; g < K; ++g) {
    for (int f = 0; f < F; ++f) o[g * (F + 1) + f] = (ACC)(ph[g * (F + 1) + f] / divisor);
    o[g * (F + 1) + F] = (ACC)bias[g];
  }
}

// 1/k for k = 0..64 (entry 0 unused), exactly rounded at compile time.
template <int... I>
struct ShapInvTable {
  double v[sizeof...(I)];
};
template <int... I>
constexpr ShapInvTable<I...> make_inv(std::integer_sequence<int, I...>) {
  return {{(I == 0 ? 0.0 : 1.0 / I)...}};
}
__constant__ ShapInvTable kShapInv = make_inv(std::make_integer_sequence<int, 65>{});

// The contrib kernel with the path arithmetic in registers.  Everything about
// a path (its length, elements, zero fractions, leaf) is the same for all 64
// lanes, so it comes through scalar loads; a lane only owns its row's one
// fractions (a bitmask: they are 0 or 1) and its path weights w[0..n], which
// stay in VGPRs because every loop that indexes them is unrolled over MAXN.
// The divisions of contrib_kernel become products with compile-time ratios
// or the 1/k table.  The row's contributions accumulate in LDS [W][64]
// (W = K * (F + 1) <= kShapLdsW), so no global read-modify-write.
constexpr int kShapLdsW = 128;
constexpr int kShapTabStride = 8;   // coefficients per one-pattern in the table (paths of <= 8 elements)
constexpr int64_t kShapWaveTarget = 65536;        // 64-row waves per contrib launch (sweep: profiles/r1_shap_sweep.log)
constexpr int64_t kShapMinPathsPerSlice = 256;
constexpr int64_t kShapMaxSlices = 64;
constexpr uint64_t kShapPartBytesMax = 2ull << 30;
// TAB: the per-element coefficients UnwoundPathSum x (one - zero) of every
// path and every pattern of one fractions were computed once per forest
// (shap_table_kernel, the same expressions in the same MT arithmetic), so a
// path costs its n element tests, n coefficient loads at [path][om] and the
// n accumulations, instead of the O(n^2) extend and unwind: the same floats.
template <typename XT, typename ACC, typename MT, int MAXN, bool TAB = false>
__global__ void __launch_bounds__(64) contrib_reg_kernel(
    const XT* __restrict__ X, int64_t rows, int64_t stride, int32_t cols, int32_t zero_map_on,
    const ShapPath* __restrict__ paths, int64_t n_paths, const ShapElem* __restrict__ elems,
    const double* __restrict__ leafv, int32_t LW, int32_t K, int32_t F, int32_t maxl,
    const double* __restrict__ bias, double divisor, double* __restrict__ part,
    int64_t paths_per_slice, ACC* __restrict__ out, const MT* __restrict__ tab,
    const int64_t* __restrict__ tab_off) {
  (void)maxl;
  extern __shared__ double shap_lds[];
  const int lane = threadIdx.x;
  const int64_t row = (int64_t)blockIdx.x * 64 + lane;
  const bool live = row < rows;
  const XT* xr = X + (live ? row : rows - 1) * stride;
  const int W = K * (F + 1);
  MT* phi = reinterpret_cast<MT*>(shap_lds) + lane;   // phi[j * 64]
  for (int j = 0; j < W; ++j) phi[j * 64] = MT(0);
  const int64_t p_begin = (int64_t)blockIdx.y * paths_per_slice;
  const int64_t p_end = p_begin + paths_per_slice < n_paths ? p_begin + paths_per_slice : n_paths;
  for (int64_t p = p_begin; p < p_end; ++p) {
    const ShapPath P = paths[p];
    const int n = P.n;
    const ShapElem* pe = elems + P.first;
    uint32_t om = 0u;                             // one fractions, bit i = element i
    for (int i = 0; i < n; ++i) {
      const ShapElem e = pe[i];
      double x = e.feature < cols ? (double)xr[e.feature] : __builtin_nan("");
      if (zero_map_on && __builtin_fabs(x) <= (double)1e-35f) x = 0.0;
      bool follow;
      if (x != x) follow = (e.flags & kShapNanOk) != 0;
      else if (x == 0.0) follow = (e.flags & kShapZeroOk) != 0;
      else follow = !(e.flags & kShapEmpty) && e.lo < x && x <= e.hi;
      om |= (follow ? 1u : 0u) << i;
    }
    if constexpr (TAB) {
      // the pattern's coefficients: kShapTabStride values, 32- or 64-byte
      // aligned, read with whole-vector loads (a lane touches one line)
      typedef MT v4_t __attribute__((ext_vector_type(4)));
      const v4_t* c4 = reinterpret_cast<const v4_t*>(tab + tab_off[p] + (int64_t)om * kShapTabStride);
      MT c[kShapTabStride];
#pragma unroll
      for (int j = 0; j < kShapTabStride / 4; ++j) {
        const v4_t v = c4[j];
        c[4 * j] = v.x;
        c[4 * j + 1] = v.y;
        c[4 * j + 2] = v.z;
        c[4 * j + 3] = v.w;
      }
      const double* lv = leafv + P.leaf * LW;
      if (LW == 1) {
        const MT l0 = static_cast<MT>(lv[0]);
#pragma unroll
        for (int e_i = 0; e_i < kShapTabStride; ++e_i)
          if (e_i < n) phi[(P.group * (F + 1) + pe[e_i].feature) * 64] += c[e_i] * l0;
      } else {
#pragma unroll
        for (int e_i = 0; e_i < kShapTabStride; ++e_i)
          if (e_i < n)
            for (int k = 0; k < LW; ++k)
              phi[(k * (F + 1) + pe[e_i].feature) * 64] += c[e_i] * static_cast<MT>(lv[k]);
      }
      continue;
    }
    // ExtendPath from scratch
    MT w[MAXN + 1];
    w[0] = MT(1);
#pragma unroll
    for (int d = 1; d <= MAXN; ++d) {
      if (d <= n) {
        const MT of = ((om >> (d - 1)) & 1u) ? MT(1) : MT(0);
        const MT zf = static_cast<MT>(pe[d - 1].zf);
        w[d] = MT(0);
#pragma unroll
        for (int i = d - 1; i >= 0; --i) {
          w[i + 1] += of * w[i] * static_cast<MT>((double)(i + 1) / (double)(d + 1));
          w[i] = zf * w[i] * static_cast<MT>((double)(d - i) / (double)(d + 1));
        }
      }
    }
    const MT rn1 = static_cast<MT>(n + 1);
    const MT in1 = static_cast<MT>(kShapInv.v[n + 1]);
    MT wn = MT(0);                              // w[n]
#pragma unroll
    for (int i = 0; i <= MAXN; ++i)
      if (i == n) wn = w[i];
    const double* lv = leafv + P.leaf * LW;
    // UnwoundPathSum per element, times (one - zero) times the leaf value
    if constexpr (std::is_same<MT, float>::value) {
      // Two elements at once in packed float32 (v_pk_mul/add_f32), both
      // branches of the unwind evaluated and selected per lane: the branch
      // on `one` diverges within a wave anyway.  Same per-element expression
      // order as the scalar loop below, so the same float results.
      typedef float f2 __attribute__((ext_vector_type(2)));
      for (int e_i = 0; e_i < n; e_i += 2) {
        const bool pair = e_i + 1 < n;
        const ShapElem ea = pe[e_i];
        const ShapElem eb = pe[pair ? e_i + 1 : e_i];
        const bool one_a = ((om >> e_i) & 1u) != 0u;
        const bool one_b = ((om >> (pair ? e_i + 1 : e_i)) & 1u) != 0u;
        const f2 zf = {static_cast<float>(ea.zf), static_cast<float>(eb.zf)};
        const f2 izf = f2{1.0f, 1.0f} / zf;
        f2 next = {wn, wn};
        f2 tot1 = {0.0f, 0.0f}, tot0 = {0.0f, 0.0f};
#pragma unroll
        for (int i = MAXN - 1; i >= 0; --i) {
          if (i < n) {
            const f2 tmp = next * (rn1 * static_cast<float>(1.0 / (double)(i + 1)));
            tot1 += tmp;
            next = w[i] - tmp * zf * (static_cast<float>(n - i) * in1);
            tot0 += w[i] * izf * (rn1 * static_cast<float>(kShapInv.v[n - i]));
          }
        }
        const float sa = (one_a ? tot1.x : tot0.x) * ((one_a ? 1.0f : 0.0f) - zf.x);
        const float sb = (one_b ? tot1.y : tot0.y) * ((one_b ? 1.0f : 0.0f) - zf.y);
        if (LW == 1) {
          const float l0 = static_cast<float>(lv[0]);
          phi[(P.group * (F + 1) + ea.feature) * 64] += sa * l0;
          if (pair) phi[(P.group * (F + 1) + eb.feature) * 64] += sb * l0;
        } else {
          for (int k = 0; k < LW; ++k) {
            const float lk = static_cast<float>(lv[k]);
            phi[(k * (F + 1) + ea.feature) * 64] += sa * lk;
            if (pair) phi[(k * (F + 1) + eb.feature) * 64] += sb * lk;
          }
        }
      }
      continue;
    }
    for (int e_i = 0; e_i < n; ++e_i) {
      const ShapElem e = pe[e_i];
      const bool one = ((om >> e_i) & 1u) != 0u;
      const MT zf = static_cast<MT>(e.zf);
      MT total = MT(0);
      if (one) {
        MT next = wn;
#pragma unroll
        for (int i = MAXN - 1; i >= 0; --i) {
          if (i < n) {
            const MT tmp = next * (rn1 * static_cast<MT>(1.0 / (double)(i + 1)));
            total += tmp;
            next = w[i] - tmp * zf * (static_cast<MT>(n - i) * in1);
          }
        }
      } else {
        const MT izf = MT(1) / zf;
#pragma unroll
        for (int i = MAXN - 1; i >= 0; --i) {
          if (i < n) total += w[i] * izf * (rn1 * static_cast<MT>(kShapInv.v[n - i]));
        }
      }
      const MT scale = total * ((one ? MT(1) : MT(0)) - zf);
      if (LW == 1) {
        phi[(P.group * (F + 1) + e.feature) * 64] += scale * static_cast<MT>(lv[0]);
      } else {
        for (int k = 0; k < LW; ++k)
          phi[(k * (F + 1) + e.feature) * 64] += scale * static_cast<MT>(lv[k]);
      }
    }
  }
  if (!live) return;
  if (part) {
    // path slice blockIdx.y: raw partial sums, [slice][W][rows] (coalesced)
    double* pp = part + (int64_t)blockIdx.y * W * rows + row;
    for (int j = 0; j < W; ++j) pp[(int64_t)j * rows] = static_cast<double>(phi[j * 64]);
    return;
  }
  ACC* o = out + row * W;
  for (int g = 0; g < K; ++g) {
    for (int f = 0; f < F; ++f)
      o[g * (F + 1) + f] = (ACC)(static_cast<double>(phi[(g * (F + 1) + f) * 64]) / divisor);
    o[g * (F + 1) + F] = (ACC)bias[g];
  }
}

// The coefficient table of contrib_reg_kernel<TAB>: one workgroup per path,
// a lane per pattern om of one fractions (bit i = element i followed): the
// path weights extended from scratch and, per element, UnwoundPathSum x
// (one - zero) -- the expressions of contrib_reg_kernel in the same order
// and type, so the table holds the floats the kernel would compute.
template <typename MT, int MAXN>
__global__ void __launch_bounds__(256) shap_table_kernel(const ShapPath* __restrict__ paths,
                                                         const ShapElem* __restrict__ elems,
                                                         const int64_t* __restrict__ tab_off,
                                                         MT* __restrict__ tab) {
  const ShapPath P = paths[blockIdx.x];
  const int n = P.n;
  const ShapElem* pe = elems + P.first;
  MT* out = tab + tab_off[blockIdx.x];
  for (uint32_t om = threadIdx.x; om < (1u << n); om += blockDim.x) {
    MT w[MAXN + 1];
    w[0] = MT(1);
#pragma unroll
    for (int d = 1; d <= MAXN; ++d) {
      if (d <= n) {
        const MT of = ((om >> (d - 1)) & 1u) ? MT(1) : MT(0);
        const MT zf = static_cast<MT>(pe[d - 1].zf);
        w[d] = MT(0);
#pragma unroll
        for (int i = d - 1; i >= 0; --i) {
          w[i + 1] += of * w[i] * static_cast<MT>((double)(i + 1) / (double)(d + 1));
          w[i] = zf * w[i] * static_cast<MT>((double)(d - i) / (double)(d + 1));
        }
      }
    }
    const MT rn1 = static_cast<MT>(n + 1);
    const MT in1 = static_cast<MT>(kShapInv.v[n + 1]);
    MT wn = MT(0);
#pragma unroll
    for (int i = 0; i <= MAXN; ++i)
      if (i == n) wn = w[i];
    for (int e_i = 0; e_i < n; ++e_i) {
      const bool one = ((om >> e_i) & 1u) != 0u;
      const MT zf = static_cast<MT>(pe[e_i].zf);
      MT total;
      if constexpr (std::is_same<MT, float>::value) {
        // contrib_reg_kernel's packed float path: both sums, then the select
        const float izf = 1.0f / zf;
        float next = wn, tot1 = 0.0f, tot0 = 0.0f;
#pragma unroll
        for (int i = MAXN - 1; i >= 0; --i) {
          if (i < n) {
            const float tmp = next * (rn1 * static_cast<float>(1.0 / (double)(i + 1)));
            tot1 += tmp;
            next = w[i] - tmp * zf * (static_cast<float>(n - i) * in1);
            tot0 += w[i] * izf * (rn1 * static_cast<float>(kShapInv.v[n - i]));
          }
        }
        total = one ? tot1 : tot0;
      } else {
        total = MT(0);
        if (one) {
          MT next = wn;
#pragma unroll
          for (int i = MAXN - 1; i >= 0; --i) {
            if (i < n) {
              const MT tmp = next * (rn1 * static_cast<MT>(1.0 / (double)(i + 1)));
              total += tmp;
              next = w[i] - tmp * zf * (static_cast<MT>(n - i) * in1);
            }
          }
        } else {
          const MT izf = MT(1) / zf;
#pragma unroll
          for (int i = MAXN - 1; i >= 0; --i) {
            if (i < n) total += w[i] * izf * (rn1 * static_cast<MT>(kShapInv.v[n - i]));
          }
        }
      }
      out[(int64_t)om * kShapTabStride + e_i] = total * ((one ? MT(1) : MT(0)) - zf);
    }
  }
}

// Sum of the path slices' partials in slice order, / divisor, bias column.
template <typename ACC>
__global__ void __launch_bounds__(256) contrib_slices_kernel(
    const double* __restrict__ part, int32_t slices, int64_t rows, int32_t K, int32_t F,
    const double* __restrict__ bias, double divisor, ACC* __restrict__ out) {
  const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= rows) return;
  const int W = K * (F + 1);
  ACC* o = out + row * W;
  for (int g = 0; g < K; ++g) {
    for (int f = 0; f < F; ++f) {
      const int j = g * (F + 1) + f;
      double t = 0.0;
      for (int sl = 0; sl < slices; ++sl) t += part[((int64_t)sl * W + j) * rows + row];
      o[j] = (ACC)(t / divisor);
    }
    o[g * (F + 1) + F] = (ACC)bias[g];
  }
}

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

int fail_hip(hipError_t e, const char* what) {
  if (e == hipSuccess) return TI_OK;
  return fail(TI_ERR_DEVICE, std::string(what) + " failed: " + hipGetErrorString(e));
}

#define TI_HIP(expr)                                                                    \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return fail(TI_ERR_DEVICE, std::string(#expr) + " failed: " + hipGetErrorString(e_)); \
  } while (0)

constexpr int kMaxHeapDepth = 8;              // deeper forests use the explicit layout
constexpr size_t kLdsPerCu = 160 * 1024;      // gfx950
constexpr size_t kFeatLdsMax = 64 * 1024;     // feature image budget per workgroup

// Environment knobs.  The layout / kernel A/B switches (TI_FORCE_LAYOUT,
// TI_TX_TOP, TI_LX_ILP, ...) are developer knobs, read only when
// TI_DEV_KNOBS=1: a serving worker that inherits a stray variable runs the
// default kernels (the reference plugin's one knob is
// nthread, python/xgbserver/xgbserver/model.py:38).  The operational settings
// below are always read; they change speed or memory, never the kernel or the
// results, and the per-forest ones are also ti_forest_set_option's.
bool dev_knobs() {
  const char* v = std::getenv("TI_DEV_KNOBS");
  return v && std::atoi(v) == 1;
}

bool operational_knob(const char* name) {
  static const char* const kOps[] = {"TI_CHUNK_MB", "TI_SHAP_TABLE_ROWS", "TI_SHAP_TABLE_MB"};
  for (const char* k : kOps)
    if (std::strcmp(k, name) == 0) return true;
  return false;
}

const char* env_knob(const char* name) {
  if (!operational_knob(name) && !dev_knobs()) return nullptr;
  const char* v = std::getenv(name);
  return v && *v ? v : nullptr;
}

int env_int(const char* name, int dflt) {
  const char* v = env_knob(name);
  return v ? std::atoi(v) : dflt;
}

// Rows per tile (= threads per workgroup) for a feature image of F columns
// of `xs`-byte elements: the largest of 256/128/64 whose [F][R] image fits
// kFeatLdsMax; 0 when even 64 rows do not fit (features read from HBM).
// (512-row tiles measured 25 % slower at F = 28: the bigger image leaves
// room for fewer workgroups per CU.)
int pick_rows(int F, size_t xs, int want) {
  if (want > 0) return want;
  for (int R = 256; R >= 64; R >>= 1)
    if (static_cast<size_t>(F) * R * xs <= kFeatLdsMax) return R;
  return 0;
}

size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

float round_down_f32(double t) {
  if (std::isnan(t)) return NAN;
  float f = static_cast<float>(t);
  if (static_cast<double>(f) > t) f = std::nextafter(f, -INFINITY);
  return f;
}

uint32_t make_meta(int32_t feature, uint8_t flags) {
  uint32_t m = static_cast<uint32_t>(feature) & ti::kMetaFeatMask;
  if (flags & TI_NODE_NAN_LEFT) m |= ti::kMetaNanLeft;
  if (flags & TI_NODE_ZERO_FLIP) m |= ti::kMetaZeroFlip;
  return m;
}

// padded heap node below a shallow leaf: always left (x <= +inf, NaN left)
constexpr uint32_t kPadMeta = ti::kMetaNanLeft;

struct DeviceForest {
  int device = -1;
  hipStream_t stream = nullptr;
  // heap layout: one record per tree, float32-input and float64-input flavours
  unsigned char* heap32 = nullptr;
  unsigned char* heap64 = nullptr;
  int32_t* heap_leaf_ids = nullptr;
  // explicit layout
  ExpNode* nodes = nullptr;
  double* thr64 = nullptr;
  int64_t* node_base = nullptr;
  int32_t* root = nullptr;
  int64_t* leaf_base = nullptr;
  void* leaves = nullptr;
  int32_t* exp_leaf_ids = nullptr;
  uint32_t* cat_words = nullptr;
  int32_t* tree_group = nullptr;
  // binned heap layout: one image + threshold tables per input dtype
  unsigned char* bh_img[2] = {nullptr, nullptr};
  unsigned char* bh_fix_img = nullptr;   // the fixed walk's permuted image (fix_permute)
  unsigned char* bh_tbl[2] = {nullptr, nullptr};
  // record layouts (6-9): rank tables per input dtype
  unsigned char* bx_tbl[2] = {nullptr, nullptr};
  // record explicit layout
  uint2* rx_recs[2] = {nullptr, nullptr};
  uint32_t* rx_base = nullptr;
  uint32_t* rx_nint = nullptr;
  int32_t* lx_stage = nullptr;
  uint32_t* tx8_pos = nullptr;   // layout 9 compact bottom: first position of each tree
  void* tx8_val = nullptr;       //   leaf value per bottom position (ACC)
  int32_t* tx8_ord = nullptr;    //   leaf ordinal per bottom position   // staged record layout (7): first tree of each stage
  uint32_t* hx_top[2] = {nullptr, nullptr};   // heap tops of layout 8, per input dtype
  // TreeSHAP path tables
  ShapPath* shap_paths = nullptr;
  ShapElem* shap_elems = nullptr;
  double* shap_leaf = nullptr;
  double* shap_bias = nullptr;
  void* shap_tab = nullptr;          // TreeSHAP coefficient table (shap_table_kernel), MT-typed
  int64_t* shap_tab_off = nullptr;   // [paths] first coefficient of each path
  std::atomic<int32_t> shap_tab_state{0};   // 0 not tried, 1 built, -1 failed or over the cap:
                                     // contributions use the extend / unwind kernel
  // ti_predict scratch: device buffers + pinned host staging (grown x2)
  void* x_buf = nullptr;
  size_t x_cap = 0;
  void* out_buf = nullptr;
  size_t out_cap = 0;
  void* hx_pin = nullptr;
  size_t hx_cap = 0;
  void* ho_pin = nullptr;
  size_t ho_cap = 0;
  // the chunk pipeline of batches larger than one chunk (predict_shard): two
  // lanes, each a stream with its own pinned and device buffers
  hipStream_t lane_stream[2] = {nullptr, nullptr};
  void* lane_hx[2] = {nullptr, nullptr};
  void* lane_ho[2] = {nullptr, nullptr};
  void* lane_dx[2] = {nullptr, nullptr};
  void* lane_do[2] = {nullptr, nullptr};
  size_t lane_x_cap = 0, lane_o_cap = 0;
  int64_t bytes = 0;
  std::mutex mu;
};

}  // namespace

struct ti_forest {
  // Forests with more than kMaxGroups outputs are split into parts of at most
  // kMaxGroups groups each (see create_chunked); the parent holds the parts.
  std::vector<std::unique_ptr<ti_forest>> parts;
  std::vector<int32_t> part_k0;                  // first output group of each part
  std::vector<std::vector<int32_t>> part_trees;  // original tree index of each part tree
  int32_t T = 0, F = 0, K = 1, LW = 1, accum = TI_F32, base_first = 1, lgb_zero_map = 0;
  int32_t zero_rule = 0, transform = TI_TRANSFORM_IDENTITY;
  double tparam = 1.0, divisor = 1.0;
  double base[ti::kMaxGroups] = {0};
  int32_t layout = 0;   // 0 heap, 1 explicit
  int32_t depth = 0;
  int64_t stride32 = 0, stride64 = 0;
  int32_t rows32 = 256, rows64 = 256;   // heap: rows per tile of each image (0 = HBM features)
  // binned heap layout (3): one image per input dtype (the ranks differ:
  // float32 view round_down_f32(t), float64 view t)
  struct BinImage {
    std::vector<unsigned char> img;   // [T][stride]
    std::vector<unsigned char> fix_img;   // img with hot pair slots first (fix_permute), or empty
    std::vector<unsigned char> tbl;   // [F][2^L] XT Eytzinger tables, or 5-ary (kary > 0)
    int32_t L = 0;
    int32_t kary = 0;                 // > 0: tbl holds float32 5-ary tables of this height
    int32_t b16 = 1;
    int32_t rows = 256;
    int32_t words = 0;                // packed bin words per row
    int64_t stride = 0;
    uint32_t mask = ti::kBNodeOffMask;   // bin-offset bits of a node word
  } bh[2];
  // record explicit layout (6): 8-byte slots per input dtype (ranks differ),
  // shared per-tree first slot, per-slot leaf values / ids
  struct RecExplicit {
    std::vector<uint2> recs;
    std::vector<unsigned char> tbl;
    int32_t L = 0;
    int32_t rows = 256;
    int32_t words = 0;
    int32_t kary = 0;            // > 0: tbl holds 5-ary search tables of this height
    int32_t b8 = 0;              // u8 bins (layout 9 only; RxBins<true> in the kernels)
    std::vector<uint32_t> top;   // heap tops (layout 8): [T][2^(hx_top+1)] u32
  } rx[2];
  std::vector<uint32_t> h_rx_base, h_rx_nint;   // h_rx_base: [T+1]
  int64_t rx_slots = 0;
  int32_t rx_ilp = 8;
  // staged record layout (7): the same records, copied into LDS a stage of
  // consecutive trees at a time; stage k holds trees [h_lx_stage[k], h_lx_stage[k+1])
  std::vector<int32_t> h_lx_stage;
  int64_t lx_stage_cap = 0;    // LDS bytes of the stage area
  int32_t lx_ilp = 8;
  // heap top + record bottom (layout 8): the top hx_top levels of each tree
  // staged in LDS hx_stage trees at a time, walked hx_ilp trees per lane
  int32_t hx_top = 0, hx_stage = 0, hx_ilp = 8;
  // heap top + staged record bottom (layout 9): per tree [top | bottom] in
  // rx[i].top, tree byte offsets [T+1] and bottom internal counts [T]; stages
  // and ILP in h_lx_stage / lx_stage_cap / lx_ilp
  std::vector<uint32_t> h_tx_off, h_tx_nint;
  // layout 9's compact u8 bottom (plan_tx8): per tree the first bottom
  // position [T+1], and per bottom position the leaf value (ACC) / ordinal
  int32_t tx8 = 0;                 // 1: compact u8 bottom, 2: compact u16 bottom, 3: the u16
                                   //   bottom walked two lanes a row (t16split_predict_kernel)
  uint32_t tx16_mask = 0;          //   u16: the bottom word's bin-offset bits (KArgs bin_mask)
  std::vector<uint32_t> h_tx8_pos;
  std::vector<unsigned char> h_tx8_val;
  std::vector<int32_t> h_tx8_ord;
  std::vector<int64_t> h_exp_src;   // explicit internal node -> descriptor node
  // TreeSHAP (TI_OUTPUT_CONTRIB); has_shap = 0 when the forest has no covers.
  // The path tables are built and uploaded on the first contributions call
  // (ensure_shap), from a host copy of the arrays they need, so predict-only
  // serving never pays for them.
  int32_t has_shap = 0, shap_maxl = 0;
  int64_t shap_npaths = 0;
  std::atomic<bool> shap_ready{false};
  std::mutex shap_mu;
  struct ShapSource {
    ti_forest_desc desc;
    std::vector<int64_t> tree_offset;
    std::vector<int32_t> tree_group, feature, left, right;
    std::vector<double> threshold, leaf_value, base_margin, cover;
    std::vector<uint8_t> flags;
  };
  std::unique_ptr<ShapSource> shap_src;
  std::vector<ShapPath> h_paths;
  // TreeSHAP coefficient table: per path, (2^n one-patterns) x n coefficients
  // (contrib_reg_kernel TAB); shap_tab_mt = 4 / 8 bytes per coefficient, 0: the
  // forest's paths cannot use one.  Built per replica on the first
  // contributions batch of at most shap_tab_rows rows, if its bytes stay under
  // shap_tab_mb (ti_forest_set_option; defaults $TI_SHAP_TABLE_ROWS /
  // $TI_SHAP_TABLE_MB read at ti_forest_create); optional: a failed build
  // leaves the extend / unwind kernel in charge.
  int32_t shap_tab_mt = 0;
  std::vector<int64_t> h_tab_off;
  int64_t shap_tab_len = 0;
  int64_t shap_tab_rows = env_int("TI_SHAP_TABLE_ROWS", 16384);
  int64_t shap_tab_mb = env_int("TI_SHAP_TABLE_MB", 1280);
  // TI_OPT_HOST_REGISTER (developer default: $TI_HOST_REGISTER under TI_DEV_KNOBS)
  std::atomic<int32_t> host_register{env_int("TI_HOST_REGISTER", 0) != 0 ? 1 : 0};
  double shap_tab_build_ms = 0.0;   // the last table build (slot's shap_table_kernel + upload)
  std::vector<ShapElem> h_elems;
  std::vector<double> h_path_leaf, h_shap_bias;
  // host images (kept until upload)
  std::vector<unsigned char> h_heap32, h_heap64;
  std::vector<int32_t> h_heap_leaf_ids;
  std::vector<ExpNode> h_nodes;
  std::vector<double> h_thr64;
  std::vector<int64_t> h_node_base, h_leaf_base;
  std::vector<int32_t> h_root, h_exp_leaf_ids, h_group;
  std::vector<uint32_t> h_cat_words;   // [nwords, w0, w1, ...] per categorical node
  int32_t has_cat = 0;
  std::vector<unsigned char> h_leaves;   // ACC-typed
  std::vector<std::unique_ptr<DeviceForest>> devs;
};

namespace {

template <typename T>
int upload(T** dst, const std::vector<T>& src, int64_t* bytes) {
  *dst = nullptr;
  if (src.empty()) return TI_OK;
  const size_t n = src.size() * sizeof(T);
  TI_HIP(hipMalloc(reinterpret_cast<void**>(dst), n));
  TI_HIP(hipMemcpy(*dst, src.data(), n, hipMemcpyHostToDevice));
  *bytes += static_cast<int64_t>(n);
  return TI_OK;
}

void free_device(DeviceForest& d) {
  if (d.device < 0) return;
  (void)hipSetDevice(d.device);
  void* ptrs[] = {d.heap32, d.heap64, d.heap_leaf_ids, d.nodes, d.thr64, d.node_base, d.root,
                  d.leaf_base, d.leaves, d.exp_leaf_ids, d.tree_group, d.x_buf, d.out_buf,
                  d.cat_words, d.bh_img[0], d.bh_img[1], d.bh_tbl[0], d.bh_tbl[1], d.bh_fix_img,
                  d.bx_tbl[0], d.bx_tbl[1],
                  d.shap_paths, d.shap_elems, d.shap_leaf, d.shap_bias, d.shap_tab, d.shap_tab_off,
                  d.rx_recs[0], d.rx_recs[1], d.rx_base, d.rx_nint, d.lx_stage,
                  d.tx8_pos, d.tx8_val, d.tx8_ord,
                  d.hx_top[0], d.hx_top[1]};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (d.hx_pin) (void)hipHostFree(d.hx_pin);
  if (d.ho_pin) (void)hipHostFree(d.ho_pin);
  d.hx_pin = d.ho_pin = nullptr;
  d.hx_cap = d.ho_cap = 0;
  for (int l = 0; l < 2; ++l) {
    if (d.lane_hx[l]) (void)hipHostFree(d.lane_hx[l]);
    if (d.lane_ho[l]) (void)hipHostFree(d.lane_ho[l]);
    if (d.lane_dx[l]) (void)hipFree(d.lane_dx[l]);
    if (d.lane_do[l]) (void)hipFree(d.lane_do[l]);
    if (d.lane_stream[l]) (void)hipStreamDestroy(d.lane_stream[l]);
    d.lane_hx[l] = d.lane_ho[l] = d.lane_dx[l] = d.lane_do[l] = nullptr;
    d.lane_stream[l] = nullptr;
  }
  d.lane_x_cap = d.lane_o_cap = 0;
  if (d.stream) (void)hipStreamDestroy(d.stream);
  d.heap32 = d.heap64 = nullptr;
  d.heap_leaf_ids = d.root = d.exp_leaf_ids = d.tree_group = nullptr;
  d.nodes = nullptr;
  d.thr64 = nullptr;
  d.node_base = d.leaf_base = nullptr;
  d.leaves = d.x_buf = d.out_buf = nullptr;
  d.cat_words = nullptr;
  for (int i = 0; i < 2; ++i) d.bh_img[i] = d.bh_tbl[i] = d.bx_tbl[i] = nullptr;
  d.bh_fix_img = nullptr;
  d.rx_recs[0] = d.rx_recs[1] = nullptr;
  d.rx_base = d.rx_nint = nullptr;
  d.lx_stage = nullptr;
  d.tx8_pos = nullptr;
  d.tx8_val = nullptr;
  d.tx8_ord = nullptr;
  d.hx_top[0] = d.hx_top[1] = nullptr;
  d.shap_paths = nullptr;
  d.shap_elems = nullptr;
  d.shap_leaf = d.shap_bias = nullptr;
  d.shap_tab = nullptr;
  d.shap_tab_off = nullptr;
  d.x_cap = d.out_cap = 0;
  d.stream = nullptr;
  d.device = -1;
}

// the TreeSHAP buffers of one replica (device current), after a failed upload
void free_shap(DeviceForest& d) {
  void* ptrs[] = {d.shap_paths, d.shap_elems, d.shap_leaf, d.shap_bias, d.shap_tab, d.shap_tab_off};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  d.shap_paths = nullptr;
  d.shap_elems = nullptr;
  d.shap_leaf = d.shap_bias = nullptr;
  d.shap_tab = nullptr;
  d.shap_tab_off = nullptr;
  d.shap_tab_state = 0;
}

// -------------------------------------------------------------- validation
int validate(const ti_forest_desc* d, std::vector<int>* depth_out) {
  if (!d) return fail(TI_ERR_INVALID, "null forest descriptor");
  if (d->abi_version != TI_ABI_VERSION)
    return fail(TI_ERR_INVALID, "abi_version mismatch: got " + std::to_string(d->abi_version));
  if (d->n_trees <= 0) return fail(TI_ERR_INVALID, "n_trees must be > 0");
  if (d->n_features <= 0 || d->n_features > (1 << 24))
    return fail(TI_ERR_INVALID, "n_features out of range");
  if (d->n_groups <= 0) return fail(TI_ERR_INVALID, "n_groups must be > 0");
  if (d->n_groups > (1 << 20)) return fail(TI_ERR_UNSUPPORTED, "n_groups > 2^20");
  if (d->leaf_width != 1 && d->leaf_width != d->n_groups)
    return fail(TI_ERR_INVALID, "leaf_width must be 1 or n_groups");
  if (d->accum_dtype != TI_F32 && d->accum_dtype != TI_F64)
    return fail(TI_ERR_INVALID, "accum_dtype must be TI_F32 or TI_F64");
  if (d->transform < TI_TRANSFORM_IDENTITY || d->transform > TI_TRANSFORM_STEP)
    return fail(TI_ERR_INVALID, "unknown transform");
  if (!(d->average_divisor > 0.0)) return fail(TI_ERR_INVALID, "average_divisor must be > 0");
  if (!d->tree_offset || !d->feature || !d->threshold || !d->flags || !d->left || !d->right ||
      !d->leaf_id || !d->leaf_value || !d->base_margin)
    return fail(TI_ERR_INVALID, "null array in forest descriptor");
  if (d->leaf_width == 1 && !d->tree_group) return fail(TI_ERR_INVALID, "null tree_group");
  if (d->tree_offset[0] != 0 || d->tree_offset[d->n_trees] != d->n_nodes)
    return fail(TI_ERR_INVALID, "tree_offset must start at 0 and end at n_nodes");
  depth_out->assign(d->n_trees, 0);
  std::vector<int> stack_node, stack_depth;
  for (int t = 0; t < d->n_trees; ++t) {
    const int64_t b = d->tree_offset[t], e = d->tree_offset[t + 1];
    if (e <= b) return fail(TI_ERR_INVALID, "tree " + std::to_string(t) + " has no nodes");
    if (e - b > (int64_t(1) << 30)) return fail(TI_ERR_INVALID, "tree too large");
    const int32_t n = static_cast<int32_t>(e - b);
    if (d->leaf_width == 1 && (d->tree_group[t] < 0 || d->tree_group[t] >= d->n_groups))
      return fail(TI_ERR_INVALID, "tree_group out of range in tree " + std::to_string(t));
    int max_depth = 0;
    int64_t visited = 0;
    stack_node.assign(1, 0);
    stack_depth.assign(1, 0);
    while (!stack_node.empty()) {
      const int v = stack_node.back(), dep = stack_depth.back();
      stack_node.pop_back();
      stack_depth.pop_back();
      if (++visited > n) return fail(TI_ERR_INVALID, "cycle in tree " + std::to_string(t));
      const int64_t g = b + v;
      if (d->feature[g] < 0) {
        max_depth = std::max(max_depth, dep);
        continue;
      }
      if (d->feature[g] >= d->n_features)
        return fail(TI_ERR_INVALID, "split feature >= n_features in tree " + std::to_string(t));
      if (d->flags[g] & TI_NODE_CATEGORICAL) {
        if (!d->cat_bits || !d->cat_offset || !d->cat_nwords)
          return fail(TI_ERR_INVALID, "categorical node without cat_bits/cat_offset/cat_nwords");
        const int64_t o = d->cat_offset[g], w = d->cat_nwords[g];
        if (o < 0 || w < 0 || o + w > d->n_cat_words)
          return fail(TI_ERR_INVALID, "categorical bitset out of range in tree " + std::to_string(t));
      }
      const int32_t l = d->left[g], r = d->right[g];
      if (l < 0 || l >= n || r < 0 || r >= n)
        return fail(TI_ERR_INVALID, "child index out of range in tree " + std::to_string(t));
      if (dep + 1 > 64) return fail(TI_ERR_UNSUPPORTED, "tree deeper than 64");
      stack_node.push_back(l);
      stack_depth.push_back(dep + 1);
      stack_node.push_back(r);
      stack_depth.push_back(dep + 1);
    }
    (*depth_out)[t] = max_depth;
  }
  return TI_OK;
}

// ------------------------------------------------------------ heap packing
template <typename XT, typename ACC>
void pack_heap(const ti_forest_desc* d, int D, int64_t stride, uint32_t feat_scale,
               std::vector<unsigned char>* img, std::vector<int32_t>* leaf_ids) {
  using Node = HeapNode<XT>;
  const int NI = (1 << D) - 1, NL = 1 << D, LW = d->leaf_width;
  img->assign(static_cast<size_t>(stride) * d->n_trees, 0);
  if (leaf_ids) leaf_ids->assign(static_cast<size_t>(NL) * d->n_trees, 0);
  struct Item { int32_t node; int32_t heap; int32_t level; };
  std::vector<Item> st;
  for (int t = 0; t < d->n_trees; ++t) {
    unsigned char* rec = img->data() + static_cast<size_t>(stride) * t;
    Node* nodes = reinterpret_cast<Node*>(rec);
    ACC* leaves = reinterpret_cast<ACC*>(rec + sizeof(Node) * NI);
    const int64_t b = d->tree_offset[t];
    st.assign(1, Item{0, 0, 0});
    while (!st.empty()) {
      const Item it = st.back();
      st.pop_back();
      const int64_t g = b + it.node;
      if (it.level == D) {   // leaf slot
        const int slot = it.heap - NI;
        for (int k = 0; k < LW; ++k)
          leaves[static_cast<size_t>(slot) * LW + k] = static_cast<ACC>(d->leaf_value[g * LW + k]);
        if (leaf_ids) (*leaf_ids)[static_cast<size_t>(t) * NL + slot] = d->leaf_id[g];
        continue;
      }
      Node nd{};
      if (d->feature[g] < 0) {   // shallow leaf: pad with always-left nodes
        nd.thr = static_cast<decltype(nd.thr)>(INFINITY);
        nd.meta = kPadMeta;
        nodes[it.heap] = nd;
        st.push_back(Item{it.node, 2 * it.heap + 1, it.level + 1});
        st.push_back(Item{it.node, 2 * it.heap + 2, it.level + 1});
      } else {
        if (sizeof(XT) == 4)
          nd.thr = static_cast<decltype(nd.thr)>(round_down_f32(d->threshold[g]));
        else
          nd.thr = static_cast<decltype(nd.thr)>(d->threshold[g]);
        nd.meta = make_meta(static_cast<int32_t>(d->feature[g] * feat_scale), d->flags[g]);
        nodes[it.heap] = nd;
        st.push_back(Item{d->left[g], 2 * it.heap + 1, it.level + 1});
        st.push_back(Item{d->right[g], 2 * it.heap + 2, it.level + 1});
      }
    }
  }
}

// -------------------------------------------------------- explicit packing
// Hot nodes first: the nodes of one tree level (tree-local indices, tree's
// first node b) ordered by cover, largest first (stable: breadth-first order
// among equals), when the model carries covers (xgboost sum_hess, LightGBM
// counts, sklearn weighted_n_node_samples) and TI_COVER_ORDER is not 0.  The
// lanes of a wave take the paths the training rows took, so at each step of a
// lockstep walk they crowd onto the high-cover nodes of a level: packed
// together, those share 128-byte lines (a gather's cost is its distinct lines:
// C4 7.3 instead of 12.5 lines a gather over N(0,1) rows, simulated) and LDS
// dwords (broadcast, not bank conflicts).  Layout only: results are unchanged.
void cover_order(const ti_forest_desc* d, int64_t b, std::vector<int32_t>* level) {
  if (!d->cover || env_int("TI_COVER_ORDER", 1) == 0) return;
  const double* c = d->cover + b;
  std::stable_sort(level->begin(), level->end(),
                   [c](int32_t x, int32_t y) { return c[x] > c[y]; });
}

// The leaves of a tree in level order, each level's by cover (cover_order):
// the leaf numbering of pack_explicit and of the record layouts' leaf slots.
void leaf_order(const ti_forest_desc* d, int64_t b, std::vector<int32_t>* out) {
  out->clear();
  std::vector<int32_t> level(1, 0), next;
  while (!level.empty()) {
    cover_order(d, b, &level);
    next.clear();
    for (const int32_t v : level) {
      const int64_t g = b + v;
      if (d->feature[g] < 0) {
        out->push_back(v);
      } else {
        next.push_back(d->left[g]);
        next.push_back(d->right[g]);
      }
    }
    level.swap(next);
  }
}

template <typename ACC>
void pack_explicit(const ti_forest_desc* d, ti_forest* f, bool leaf_ids_only) {
  const int LW = d->leaf_width;
  f->h_nodes.clear();
  f->h_thr64.clear();
  f->h_exp_src.clear();
  f->h_node_base.assign(d->n_trees, 0);
  f->h_leaf_base.assign(d->n_trees, 0);
  f->h_root.assign(d->n_trees, 0);
  f->h_exp_leaf_ids.clear();
  f->h_cat_words.clear();
  std::vector<ACC> leaves;
  std::vector<int32_t> remap;
  std::vector<int32_t> queue, lorder;
  for (int t = 0; t < d->n_trees; ++t) {
    const int64_t b = d->tree_offset[t];
    const int32_t n = static_cast<int32_t>(d->tree_offset[t + 1] - b);
    remap.assign(n, 0);
    const int64_t nb = static_cast<int64_t>(f->h_nodes.size());
    const int64_t lb = static_cast<int64_t>(f->h_exp_leaf_ids.size());
    f->h_node_base[t] = nb;
    f->h_leaf_base[t] = lb;
    // leaves numbered level by level, the level's by cover (leaf_order: the
    // record layouts' leaf slots follow the same order, so one leaf table
    // serves every layout); internal nodes breadth-first: the top levels of a
    // tree share cache lines
    leaf_order(d, b, &lorder);
    for (size_t i = 0; i < lorder.size(); ++i) {
      const int64_t g = b + lorder[i];
      remap[lorder[i]] = ~static_cast<int32_t>(i);
      f->h_exp_leaf_ids.push_back(d->leaf_id[g]);
      if (!leaf_ids_only)
        for (int k = 0; k < LW; ++k) leaves.push_back(static_cast<ACC>(d->leaf_value[g * LW + k]));
    }
    queue.assign(1, 0);
    int32_t n_int = 0;
    for (size_t qi = 0; qi < queue.size(); ++qi) {
      const int32_t v = queue[qi];
      const int64_t g = b + v;
      if (d->feature[g] < 0) continue;
      remap[v] = n_int++;
      queue.push_back(d->left[g]);
      queue.push_back(d->right[g]);
    }
    f->h_nodes.resize(nb + n_int);
    f->h_thr64.resize(nb + n_int);
    f->h_exp_src.resize(nb + n_int);
    for (size_t qi = 0; qi < queue.size(); ++qi) {
      const int32_t v = queue[qi];
      const int64_t g = b + v;
      if (d->feature[g] < 0) continue;
      ExpNode e;
      e.thr = round_down_f32(d->threshold[g]);
      e.meta = make_meta(d->feature[g], d->flags[g]);
      if (d->flags[g] & TI_NODE_CATEGORICAL) {
        // threshold slot carries the word offset of [nwords, bitset...]
        const uint32_t at = static_cast<uint32_t>(f->h_cat_words.size());
        const int32_t nw = d->cat_nwords[g];
        f->h_cat_words.push_back(static_cast<uint32_t>(nw));
        for (int32_t w = 0; w < nw; ++w) f->h_cat_words.push_back(d->cat_bits[d->cat_offset[g] + w]);
        std::memcpy(&e.thr, &at, sizeof(at));
        e.meta = (static_cast<uint32_t>(d->feature[g]) & ti::kMetaFeatMask) | ti::kMetaCat;
      }
      e.left = remap[d->left[g]];
      e.right = remap[d->right[g]];
      f->h_nodes[nb + remap[v]] = e;
      f->h_thr64[nb + remap[v]] = d->threshold[g];
      f->h_exp_src[nb + remap[v]] = g;
    }
    f->h_root[t] = remap[0];
  }
  if (leaf_ids_only) {
    f->h_nodes.clear();
    f->h_thr64.clear();
    f->h_node_base.clear();
    f->h_root.clear();
    return;
  }
  f->h_leaves.resize(leaves.size() * sizeof(ACC));
  if (!leaves.empty()) std::memcpy(f->h_leaves.data(), leaves.data(), f->h_leaves.size());
}


// ------------------------------------------------------ binned heap packing
// Rank binning (treeinfer_kernels.h, stage_bins): per feature the sorted
// distinct thresholds of the XT view, an Eytzinger search table of 2^L
// entries (1-based, +inf padded) and per-node ranks.  Returns false when the
// forest does not qualify (too many distinct thresholds, or a feature image
// whose offsets overflow the node's 15 bits even at 64-row tiles).
template <typename XT>
XT threshold_view(double t) {
  if (sizeof(XT) == 4) return static_cast<XT>(round_down_f32(t));
  return static_cast<XT>(t);
}

void eytzinger_fill(const std::vector<double>& sorted, std::vector<double>* out, size_t k, size_t* i) {
  if (k >= out->size()) return;
  eytzinger_fill(sorted, out, 2 * k, i);
  (*out)[k] = *i < sorted.size() ? sorted[*i] : INFINITY;
  ++*i;
  eytzinger_fill(sorted, out, 2 * k + 1, i);
}

// Per-feature rank tables of one XT view.  With zero_bins, every feature
// that a LightGBM zero-missing node tests also gets the thresholds {-denorm_min,
// 0}: then exactly x == 0 (+-0) falls in the bin 1 + index(0) (zbin), so the
// zero rule becomes an integer compare as well.
template <typename XT>
struct RankTables {
  std::vector<std::vector<XT>> u;   // sorted distinct thresholds per feature
  std::vector<uint32_t> zbin;       // bin of exact 0 per feature (0: none)
  size_t m_max = 0;
  int L = 0;

  uint32_t rank(int f, double thr) const {
    const XT t = threshold_view<XT>(thr);
    if (std::isnan(static_cast<double>(t))) return 0;   // NaN threshold: never left
    return 1u + static_cast<uint32_t>(std::lower_bound(u[f].begin(), u[f].end(), t) - u[f].begin());
  }
};

template <typename XT>
RankTables<XT> collect_ranks(const ti_forest_desc* d, bool zero_bins) {
  RankTables<XT> rt;
  const int F = d->n_features;
  rt.u.assign(F, {});
  rt.zbin.assign(F, 0);
  std::vector<char> zf(F, 0);
  for (int64_t g = 0; g < d->n_nodes; ++g) {
    if (d->feature[g] < 0 || (d->flags[g] & TI_NODE_CATEGORICAL)) continue;
    const XT t = threshold_view<XT>(d->threshold[g]);
    if (!std::isnan(static_cast<double>(t))) rt.u[d->feature[g]].push_back(t);
    if (zero_bins && (d->flags[g] & TI_NODE_ZERO_FLIP)) zf[d->feature[g]] = 1;
  }
  for (int f = 0; f < F; ++f) {
    auto& v = rt.u[f];
    if (zf[f]) {
      v.push_back(XT(0));
      v.push_back(-std::numeric_limits<XT>::denorm_min());
    }
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    rt.m_max = std::max(rt.m_max, v.size());
    if (zf[f]) rt.zbin[f] = 1u + static_cast<uint32_t>(std::lower_bound(v.begin(), v.end(), XT(0)) - v.begin());
  }
  while ((static_cast<size_t>(1) << rt.L) - 1 < rt.m_max) ++rt.L;
  return rt;
}

// [F][2^L] Eytzinger search tables (1-based, +inf padded) as XT bytes.
template <typename XT>
void eytzinger_tables(const RankTables<XT>& rt, std::vector<unsigned char>* out) {
  const int F = static_cast<int>(rt.u.size());
  const size_t tsz = static_cast<size_t>(1) << rt.L;
  out->assign(static_cast<size_t>(F) * tsz * sizeof(XT), 0);
  XT* tbl = reinterpret_cast<XT*>(out->data());
  std::vector<double> srt, ey(tsz);
  for (int f = 0; f < F; ++f) {
    srt.assign(rt.u[f].begin(), rt.u[f].end());
    size_t i = 0;
    std::fill(ey.begin(), ey.end(), static_cast<double>(INFINITY));
    eytzinger_fill(srt, &ey, 1, &i);
    for (size_t k = 0; k < tsz; ++k) tbl[f * tsz + k] = static_cast<XT>(ey[k]);
  }
}

// 5-ary search tables (float32 view of layouts 6-9, rx_stage_bins): per
// feature a complete 5-ary tree of height H, node j (0-based, children
// 5j+1 .. 5j+5) holding 4 keys, filled in order with the sorted thresholds and
// +inf padding.  The search counts the keys below x at each node and descends;
// after H levels, j - (5^H - 1)/4 = #{u < x}: the same rank as the Eytzinger
// search, in H 16-byte gathers instead of L 4-byte ones.
template <typename XT>
void kary_fill(const std::vector<XT>& srt, std::vector<XT>* out, size_t j, int level, int H,
               size_t* i) {
  if (level == H) return;
  for (int c = 0; c < 4; ++c) {
    kary_fill(srt, out, 5 * j + 1 + c, level + 1, H, i);
    (*out)[4 * j + c] = *i < srt.size() ? srt[*i] : static_cast<XT>(INFINITY);
    ++*i;
  }
  kary_fill(srt, out, 5 * j + 5, level + 1, H, i);
}

// (float32 view: 16-byte nodes; float64 view: 32-byte nodes of 4 doubles)
template <typename XT>
void kary_tables(const RankTables<XT>& rt, std::vector<unsigned char>* out, int* height) {
  const int F = static_cast<int>(rt.u.size());
  int H = 1;
  size_t p5 = 5;
  while (p5 - 1 < rt.m_max) {
    p5 *= 5;
    ++H;
  }
  const size_t nn = (p5 - 1) / 4;
  out->assign(static_cast<size_t>(F) * nn * 4 * sizeof(XT), 0);
  std::vector<XT> node(nn * 4), srt;
  for (int f = 0; f < F; ++f) {
    srt.assign(rt.u[f].begin(), rt.u[f].end());
    size_t i = 0;
    kary_fill(srt, &node, 0, 0, H, &i);
    std::memcpy(out->data() + static_cast<size_t>(f) * nn * 4 * sizeof(XT), node.data(),
                nn * 4 * sizeof(XT));
  }
  *height = H;
}

// The fixed walk (bheap_fix_kernel) finds a node's children pair through the
// pair slot the node word carries in bits 3..10, not by heap arithmetic, so
// within a level the slots may be any permutation.  fix_permute numbers each
// level's nodes by cover, largest first: the lanes of a wave, which crowd onto
// the nodes the training rows took, then read pairs packed at the start of the
// level's slots -- the same address (a broadcast) or nearby dwords -- instead
// of pairs up to 1 KB apart whose dwords collide in the LDS banks.  Same
// words, same walk, same sums; only the fixed walk reads this image (leaf ids
// keep the heap-indexed walk on img).
void fix_permute(ti_forest::BinImage* bi, const std::vector<double>& hcov, int NE) {
  const int64_t T = static_cast<int64_t>(bi->img.size()) / bi->stride;
  bi->fix_img.assign(bi->img.size(), 0);
  std::vector<int32_t> pi(NE, 0), lvl;
  for (int64_t t = 0; t < T; ++t) {
    const uint32_t* on = reinterpret_cast<const uint32_t*>(bi->img.data() + bi->stride * t);
    const float* ol = reinterpret_cast<const float*>(on + NE);
    uint32_t* nn = reinterpret_cast<uint32_t*>(bi->fix_img.data() + bi->stride * t);
    float* nl = reinterpret_cast<float*>(nn + NE);
    const double* c = hcov.data() + static_cast<size_t>(t) * NE;
    for (int lo = 1; lo < NE; lo <<= 1) {   // level [lo, 2 lo): slots by cover
      lvl.resize(lo);
      for (int i = 0; i < lo; ++i) lvl[i] = lo + i;
      std::stable_sort(lvl.begin(), lvl.end(), [c](int32_t x, int32_t y) { return c[x] > c[y]; });
      for (int i = 0; i < lo; ++i) pi[lvl[i]] = lo + i;
    }
    auto relabel = [&](uint32_t w, int h) { return (w & ~0x7F8u) | (static_cast<uint32_t>(pi[h]) << 3); };
    nn[1] = relabel(on[1], 1);
    for (int v = 1; v < NE; ++v)
      for (int s = 0; s < 2; ++s) {
        const int ch = 2 * v + s, nw = 2 * pi[v] + s;
        if (ch < NE) nn[nw] = relabel(on[ch], ch);
        else nl[nw - NE] = ol[ch - NE];
      }
  }
}

template <typename XT, typename ACC>
bool pack_bheap(const ti_forest_desc* d, int D, ti_forest::BinImage* bi,
                std::vector<int32_t>* leaf_ids) {
  const int F = d->n_features;
  const int LW = d->leaf_width;
  const RankTables<XT> rt = collect_ranks<XT>(d, false);
  const size_t m_max = rt.m_max;
  if (m_max > 65533) return false;
  bi->b16 = m_max > 253 ? 1 : 0;
  const int P = bi->b16 ? 2 : 4;
  bi->words = (F + P - 1) / P;
  // 512: measured +5% over 256 at F = 28 (32 waves/CU); a power of two in
  // [64, 512], as pack_rexplicit (the lane part is OR-ed into the offset)
  int R = 64;
  while (R < 512 && 2 * R <= env_int("TI_BHEAP_ROWS", 512)) R *= 2;
  while (R > 64 && static_cast<int64_t>(bi->words) * R * 4 > static_cast<int64_t>(ti::kBNodeOffMask) + 1)
    R >>= 1;
  if (static_cast<int64_t>(bi->words) * R * 4 > static_cast<int64_t>(ti::kBNodeOffMask) + 1) return false;
  bi->rows = R;
  bi->L = rt.L;
  bi->kary = 0;
  if constexpr (sizeof(XT) == 4) {
    if (env_int("TI_KARY", 1) != 0) kary_tables(rt, &bi->tbl, &bi->kary);
    else eytzinger_tables(rt, &bi->tbl);
  } else {
    eytzinger_tables(rt, &bi->tbl);
  }
  // 512-row tiles: the offset bits are 0, 1 and 11..14, and each node word
  // also carries its own heap index in bits 3..10 (the fixed-layout walk's
  // pair address; treeinfer_kernels.h, kBNodeOffMask512)
  const bool with_index = R == 512;
  bi->mask = with_index ? ti::kBNodeOffMask512 : ti::kBNodeOffMask;
  auto node_word = [&](int64_t g) -> uint32_t {
    const int f = d->feature[g];
    const uint32_t rank = rt.rank(f, d->threshold[g]);
    const uint32_t off = static_cast<uint32_t>((f / P) * R * 4 + (f % P) * (4 / P));
    uint32_t w = off | (rank << 16);
    if (d->flags[g] & TI_NODE_NAN_LEFT) w |= ti::kBNodeNanLeft;
    return w;
  };
  const int NE = 1 << D;
  bi->stride = static_cast<int64_t>(align16(sizeof(uint32_t) * NE + sizeof(ACC) * NE * LW));
  bi->img.assign(static_cast<size_t>(bi->stride) * d->n_trees, 0);
  if (leaf_ids) leaf_ids->assign(static_cast<size_t>(NE) * d->n_trees, 0);
  struct Item { int32_t node; int32_t heap; int32_t level; double cov; };
  std::vector<Item> st;
  // the fixed walk's permuted image (fix_permute): float32 view, 512-row
  // tiles, depth-8 records of float leaves, covers in the model
  const bool perm = sizeof(XT) == 4 && sizeof(ACC) == 4 && with_index && D == 8 && LW == 1 && d->cover &&
                    env_int("TI_FIX_PERM", 1) != 0;
  std::vector<double> hcov(perm ? static_cast<size_t>(NE) * d->n_trees : 0, 0.0);
  for (int t = 0; t < d->n_trees; ++t) {
    unsigned char* rec = bi->img.data() + static_cast<size_t>(bi->stride) * t;
    uint32_t* nodes = reinterpret_cast<uint32_t*>(rec);
    ACC* leaves = reinterpret_cast<ACC*>(rec + sizeof(uint32_t) * NE);
    const int64_t b = d->tree_offset[t];
    st.assign(1, Item{0, 1, 0, d->cover ? d->cover[b] : 0.0});
    while (!st.empty()) {
      const Item it = st.back();
      st.pop_back();
      const int64_t g = b + it.node;
      if (perm && it.level < D) hcov[static_cast<size_t>(t) * NE + it.heap] = it.cov;
      if (it.level == D) {
        const int slot = it.heap - NE;
        for (int k = 0; k < LW; ++k)
          leaves[static_cast<size_t>(slot) * LW + k] = static_cast<ACC>(d->leaf_value[g * LW + k]);
        if (leaf_ids) (*leaf_ids)[static_cast<size_t>(t) * NE + slot] = d->leaf_id[g];
        continue;
      }
      const uint32_t idx = with_index ? static_cast<uint32_t>(it.heap) << 3 : 0u;
      if (d->feature[g] < 0) {   // shallow leaf: always-left padding down to level D
        nodes[it.heap] = (0xFFFFu << 16) | idx;
        st.push_back(Item{it.node, 2 * it.heap, it.level + 1, it.cov});
        st.push_back(Item{it.node, 2 * it.heap + 1, it.level + 1, 0.0});
      } else {
        nodes[it.heap] = node_word(g) | idx;
        st.push_back(Item{d->left[g], 2 * it.heap, it.level + 1,
                          d->cover ? d->cover[b + d->left[g]] : 0.0});
        st.push_back(Item{d->right[g], 2 * it.heap + 1, it.level + 1,
                          d->cover ? d->cover[b + d->right[g]] : 0.0});
      }
    }
  }
  if (perm) fix_permute(bi, hcov, NE);
  return true;
}

// ------------------------------------------------ record explicit packing
// Slots of layout 6 (treeinfer_kernels.h, rx_walk): per tree the internal
// nodes breadth-first in [0, nint), then the leaves in the same breadth-first
// order as pack_explicit numbers them (so leaf ids / vector leaves share its
// tables), n slots for n nodes.  Returns false when a tree has more than
// 65,535 nodes (16-bit child slots).
bool plan_rx_slots(const ti_forest_desc* d, ti_forest* f, std::vector<uint32_t>* slot_of) {
  std::vector<int32_t> level, next;
  slot_of->assign(d->n_nodes, 0);
  f->h_rx_base.assign(d->n_trees + 1, 0);   // [T]: the slot count (staged layout)
  f->h_rx_nint.assign(d->n_trees, 0);
  if (d->n_nodes >= (int64_t(1) << 31)) return false;
  std::vector<int32_t> q;
  for (int t = 0; t < d->n_trees; ++t) {
    const int64_t b = d->tree_offset[t];
    const int64_t n = d->tree_offset[t + 1] - b;
    if (n > 65535) return false;
    f->h_rx_base[t] = static_cast<uint32_t>(b);   // a tree takes as many slots as nodes
    // level by level (the lockstep walks gather one level per step), and
    // within a level the internal nodes of largest cover first (cover_order)
    level.assign(1, 0);
    uint32_t n_int = 0;
    while (!level.empty()) {
      cover_order(d, b, &level);
      next.clear();
      for (const int32_t v : level) {
        const int64_t g = b + v;
        if (d->feature[g] < 0) continue;
        (*slot_of)[g] = n_int++;
        next.push_back(d->left[g]);
        next.push_back(d->right[g]);
      }
      level.swap(next);
    }
    // leaves in pack_explicit's numbering (leaf ids and vector leaves are
    // found as leaf_base + slot - nint): leaf_order
    leaf_order(d, b, &q);
    for (size_t i = 0; i < q.size(); ++i) (*slot_of)[b + q[i]] = n_int + static_cast<uint32_t>(i);
    f->h_rx_nint[t] = n_int;
  }
  f->h_rx_base[d->n_trees] = static_cast<uint32_t>(d->n_nodes);
  f->rx_slots = d->n_nodes;
  return true;
}

// Records of one input view (ranks differ between the float32 and float64
// views).  Returns false when the bins do not fit u16 (more than 65,533
// distinct thresholds on a feature; 16,382 for zero-missing forests, whose
// bins are doubled) or, with b8, u8 (254; 126 with the zero rule: NaN is bin
// 0, values 1 .. m + 1), or the bin image does not fit 64 KB at 64-row tiles.
// u8 images hold four bins a word, so a tile of twice the rows (512,
// TI_RX_ROWS8) fits the LDS a u16 tile of 256 takes: 4 waves per SIMD
// instead of 2 at C3's 100 features.
template <typename XT, typename ACC>
bool pack_rexplicit(const ti_forest_desc* d, const ti_forest* f,
                    const std::vector<uint32_t>& slot_of, ti_forest::RecExplicit* rx,
                    bool b8 = false) {
  const bool zero = f->zero_rule != 0;
  const RankTables<XT> rt = collect_ranks<XT>(d, zero);
  if (rt.m_max > (b8 ? (zero ? 126u : 254u) : (zero ? 16382u : 65533u))) return false;
  const int P = b8 ? 4 : 2;   // bins per word
  rx->b8 = b8 ? 1 : 0;
  rx->words = (d->n_features + P - 1) / P;
  const uint32_t nan_left = b8 ? ti::RxBins<true>::kNanLeft : ti::kRxNanLeft;
  const uint32_t zero_flip = b8 ? ti::RxBins<true>::kZeroFlip : ti::kRxZeroFlip;
  // a power of two in [64, 512]: the kernels OR the lane part (tid * 4) into
  // the feature's word offset (word * R * 4), which holds only then
  int R = 64;
  const int want_rows = b8 ? env_int("TI_RX_ROWS8", 512) : env_int("TI_RX_ROWS", 256);
  while (R < 512 && 2 * R <= want_rows) R *= 2;
  while (R > 64 && static_cast<size_t>(rx->words) * R * 4 > kFeatLdsMax) R >>= 1;
  if (static_cast<size_t>(rx->words) * R * 4 > kFeatLdsMax) return false;
  rx->rows = R;
  rx->L = rt.L;
  rx->kary = 0;
  // 5-ary tables for both views (float64: TI_KARY64, 32-byte nodes)
  if (env_int(sizeof(XT) == 4 ? "TI_KARY" : "TI_KARY64", 1) != 0) kary_tables(rt, &rx->tbl, &rx->kary);
  else eytzinger_tables(rt, &rx->tbl);
  // an even slot count: the staged layout copies whole 16-byte words
  rx->recs.assign(d->n_nodes + (d->n_nodes & 1), uint2{0u, 0u});
  const bool scalar_leaves = d->leaf_width == 1;
  for (int t = 0; t < d->n_trees; ++t) {
    const int64_t b = d->tree_offset[t];
    for (int64_t g = b; g < d->tree_offset[t + 1]; ++g) {
      uint2 r{0u, 0u};
      if (d->feature[g] < 0) {
        if (scalar_leaves) {
          const ACC v = static_cast<ACC>(d->leaf_value[g]);
          std::memcpy(&r, &v, sizeof(ACC));
        }
      } else {
        const int fe = d->feature[g];
        const uint32_t off = static_cast<uint32_t>((fe / P) * R * 4 + (fe % P) * (4 / P));
        const uint32_t rank = rt.rank(fe, d->threshold[g]);
        r.x = off | ((d->flags[g] & TI_NODE_NAN_LEFT) ? nan_left : 0u);
        if (zero) {
          r.x |= (2u * rank + 1u) << 16;   // <= 32,765: bit 31 stays clear
          if (d->flags[g] & TI_NODE_ZERO_FLIP) r.x |= zero_flip;
        } else {
          r.x |= rank << 16;
        }
        r.y = (slot_of[b + d->right[g]] << 16) | slot_of[b + d->left[g]];
      }
      rx->recs[b + slot_of[g]] = r;
    }
  }
  return true;
}

// Staged record layout (7): forests whose trees are small enough that a run
// of several consecutive trees' records fits in LDS beside the bin image walk
// from LDS instead of gathering every node through the vector memory pipe
// (the bound of layout 6: TD busy 92 % of the kernel, profiles/r2_c3_l6b_*).
// The stage area is what 160 KB / TI_LX_WGS (2) workgroups per CU leave after
// the bin image, capped by the prefetch registers (kLxPf x 16 B per thread).
// A stage is a maximal run of consecutive trees whose records (their span
// widened to 16-byte words) fit the area.  Returns false (layout 6 stays) when
// fewer than two of the largest trees fit.
constexpr int kLxPf = 8;
// every masked bin address ((x & 0xFFFA) | lane offset <= 66,558) must stay
// inside the workgroup's LDS allocation: leaf records hold values, not offsets
constexpr size_t kLxMinLds = 66560;
bool plan_lx_stages(ti_forest* f, int T) {
  const int R = f->rx[0].rows;
  if (f->rx[1].rows != R) return false;
  const size_t bins = align16(static_cast<size_t>(std::max(f->rx[0].words, f->rx[1].words)) * R * 4 + 4);
  const int wgs = std::max(1, env_int("TI_LX_WGS", 2));
  size_t cap = kLdsPerCu / static_cast<size_t>(wgs);
  cap = cap > bins ? cap - bins : 0;
  cap = std::min(cap, static_cast<size_t>(kLxPf) * 16 * R) & ~size_t(15);
  const std::vector<uint32_t>& b = f->h_rx_base;
  auto span = [&](int t0, int t1) {
    return ((static_cast<size_t>(b[t1]) * 8 + 15) & ~size_t(15)) - ((static_cast<size_t>(b[t0]) * 8) & ~size_t(15));
  };
  size_t biggest = 0;
  for (int t = 0; t < T; ++t) biggest = std::max(biggest, span(t, t + 1));
  if (T < 2 || cap < 2 * biggest + 16) return false;
  f->h_lx_stage.assign(1, 0);
  int t0 = 0;
  while (t0 < T) {
    int t1 = t0 + 1;
    while (t1 < T && span(t0, t1 + 1) <= cap) ++t1;
    f->h_lx_stage.push_back(t1);
    t0 = t1;
  }
  f->lx_stage_cap = static_cast<int64_t>(cap);
  // children as byte offsets in the tree (a stage is <= 32 KB: < 8,192 slots)
  for (auto& rx : f->rx)
    for (int t = 0; t < T; ++t)
      for (uint32_t v = b[t]; v < b[t] + f->h_rx_nint[t]; ++v) {
        uint2& r = rx.recs[v];
        r.y = (((r.y >> 16) << 3) << 16) | ((r.y & 0xFFFFu) << 3);
      }
  // trees in lockstep per lane: a stage's worth when stages hold 7 or 8 trees
  // (C3: 7 trees of 4,072 B per 30.7 KB stage; a group wider than the stage
  // walks a duplicate tree), else 4
  const double per_stage = static_cast<double>(T) / static_cast<double>(f->h_lx_stage.size() - 1);
  f->lx_ilp = per_stage >= 7.5 ? 8 : per_stage >= 6.5 ? 7 : 4;
  const int force_ilp = env_int("TI_LX_ILP", 0);
  if (force_ilp > 0) f->lx_ilp = force_ilp >= 8 ? 8 : force_ilp == 7 ? 7 : 4;
  return true;
}

// Heap tops of layout 8 (treeinfer_kernels.h, hexplicit_predict_kernel): per
// tree 2^(D0+1) u32 entries -- [0] unused, [1, 2^D0) the x words of layout
// 6's records at the heap positions of the top D0 levels (padding below a
// shallow leaf: rank 0xFFFF, NaN-left, which goes left on every bin), then at
// [2^D0, 2^(D0+1)) the layout-6 slot where the walk continues: the node at
// depth D0, or the leaf that ended the path above it.
constexpr uint32_t kHxPad = 0xFFFF0000u | ti::kRxNanLeft;
constexpr uint32_t kHxPad8 = 0xFFFF0000u | ti::RxBins<true>::kNanLeft;   // u8 bins (layout 9)
constexpr int kHxPf = 8;   // = PF of hexplicit_predict_kernel
void pack_htop(const ti_forest_desc* d, const std::vector<uint32_t>& slot_of, int D0,
               ti_forest::RecExplicit* rx) {
  const size_t NE = size_t(1) << D0;
  rx->top.assign(static_cast<size_t>(d->n_trees) * 2 * NE, 0u);
  struct Item { int32_t v; uint32_t p; int l; };
  std::vector<Item> st;
  for (int t = 0; t < d->n_trees; ++t) {
    const int64_t b = d->tree_offset[t];
    uint32_t* top = &rx->top[static_cast<size_t>(t) * 2 * NE];
    st.assign(1, Item{0, 1u, 0});
    while (!st.empty()) {
      const Item it = st.back();
      st.pop_back();
      const int64_t g = b + it.v;
      if (it.l == D0) {
        top[it.p] = slot_of[g];
        continue;
      }
      const bool leaf = d->feature[g] < 0;
      top[it.p] = leaf ? kHxPad : rx->recs[b + slot_of[g]].x;
      st.push_back(Item{leaf ? it.v : d->left[g], 2 * it.p, it.l + 1});
      st.push_back(Item{leaf ? it.v : d->right[g], 2 * it.p + 1, it.l + 1});
    }
  }
}

// Layout 8's parameters and images: the top depth D0 (TI_HX_TOP, default 8,
// at most the forest depth), ILP trees per lane (TI_HX_ILP: 4 or 8) and the
// stage (TI_HX_STAGE trees, default ILP; at most what the prefetch registers
// carry and what leaves the bin image room in 160 KB).  Falls back to layout 6
// (returns false) when even ILP tops do not fit.
constexpr int kHxMinDepth = 12;
// layout 8's top depth for a forest of depth D (TI_HX_TOP, default 8)
int hx_top_depth(int D) {
  return std::max(1, std::min(env_int("TI_HX_TOP", 8), std::min(D, 12)));
}
bool plan_htop(const ti_forest_desc* d, ti_forest* f, const std::vector<uint32_t>& slot_of, int D) {
  const int D0 = hx_top_depth(D);
  const int ilp = env_int("TI_HX_ILP", 8) >= 8 ? 8 : 4;
  const int R = f->rx[0].rows;
  if (f->rx[1].rows != R) return false;
  const size_t stride = static_cast<size_t>(8) << D0;
  const size_t bins = align16(static_cast<size_t>(std::max(f->rx[0].words, f->rx[1].words)) * R * 4 + 4);
  const size_t cap = std::min(static_cast<size_t>(kHxPf) * 16 * R, kLdsPerCu > bins ? kLdsPerCu - bins : 0);
  int S = env_int("TI_HX_STAGE", ilp);
  S = std::max(1, std::min<int>(S, f->T));
  while (S > 1 && S * stride > cap) --S;
  if (S * stride > cap || S < std::min(ilp, f->T)) return false;
  for (auto& rx : f->rx) pack_htop(d, slot_of, D0, &rx);
  f->hx_top = D0;
  f->hx_ilp = ilp;
  f->hx_stage = S;
  f->layout = 8;
  return true;
}

// Layout 9 (treeinfer_kernels.h, texplicit_predict_kernel): per tree, a heap
// top of D0 levels (as layout 8's, the entries at [2^D0, 2^(D0+1)) holding
// byte offsets into the bottom) and the bottom: layout 6's records from the
// first internal node at depth >= D0 on (breadth-first order puts the top's
// internal nodes first), children rebased to byte offsets from the bottom's
// start, padded to 16 bytes.  Stages as layout 7's.  Returns false (the
// caller keeps its choice) when two of the largest trees do not fit a stage
// or a bottom exceeds 16-bit byte offsets.
bool plan_tx(const ti_forest_desc* d, ti_forest* f, const std::vector<uint32_t>& slot_of, int D) {
  int D0 = env_int("TI_TX_TOP", 6);
  D0 = std::max(1, std::min(D0, std::min(D, 10)));
  const int T = d->n_trees;
  const size_t NE = size_t(1) << D0;
  const uint32_t topb = static_cast<uint32_t>(8 * NE);
  std::vector<int32_t> dep, q;
  std::vector<uint32_t> ntop(T), nslots(T);
  f->h_tx_off.assign(T + 1, 0);
  f->h_tx_nint.assign(T, 0);
  for (int t = 0; t < T; ++t) {
    const int64_t b = d->tree_offset[t];
    const int32_t n = static_cast<int32_t>(d->tree_offset[t + 1] - b);
    dep.assign(n, 0);
    q.assign(1, 0);
    uint32_t nt = 0;
    for (size_t qi = 0; qi < q.size(); ++qi) {
      const int32_t v = q[qi];
      const int64_t g = b + v;
      if (d->feature[g] < 0) continue;
      if (dep[v] < D0) ++nt;
      dep[d->left[g]] = dep[d->right[g]] = dep[v] + 1;
      q.push_back(d->left[g]);
      q.push_back(d->right[g]);
    }
    ntop[t] = nt;
    nslots[t] = static_cast<uint32_t>(n) - nt;
    if (static_cast<size_t>(nslots[t]) * 8 > 65528) {
      f->h_tx_off.clear();
      f->h_tx_nint.clear();
      return false;
    }
    f->h_tx_nint[t] = f->h_rx_nint[t] - nt;
    const uint64_t end = f->h_tx_off[t] + topb + ((static_cast<uint64_t>(nslots[t]) * 8 + 15) & ~uint64_t(15));
    if (end > 0xFFFFFFF0ull) {
      f->h_tx_off.clear();
      f->h_tx_nint.clear();
      return false;
    }
    f->h_tx_off[t + 1] = static_cast<uint32_t>(end);
  }
  // stages: as plan_lx_stages
  const int R = f->rx[0].rows;
  if (f->rx[1].rows != R) return false;
  const size_t bins = align16(static_cast<size_t>(std::max(f->rx[0].words, f->rx[1].words)) * R * 4 + 4);
  const int wgs = std::max(1, env_int("TI_LX_WGS", 2));
  size_t cap = kLdsPerCu / static_cast<size_t>(wgs);
  cap = cap > bins ? cap - bins : 0;
  cap = std::min(cap, static_cast<size_t>(kLxPf) * 16 * R) & ~size_t(15);
  const std::vector<uint32_t>& o = f->h_tx_off;
  size_t biggest = 0;
  for (int t = 0; t < T; ++t) biggest = std::max<size_t>(biggest, o[t + 1] - o[t]);
  if (T < 2 || cap < 2 * biggest) {
    f->h_tx_off.clear();
    f->h_tx_nint.clear();
    return false;
  }
  // TI_LX_ILP > 0 also cuts stages to whole groups of that many trees
  // (plan_tx8 always does; here the default ILP follows the stage size)
  const int force_ilp = env_int("TI_LX_ILP", 0);
  const int cut = force_ilp > 0 ? (force_ilp >= 8 ? 8 : force_ilp == 7 ? 7 : 4) : 0;
  std::vector<int32_t> stages(1, 0);
  int t0 = 0;
  while (t0 < T) {
    int t1 = t0 + 1;
    while (t1 < T && o[t1 + 1] - o[t0] <= cap) ++t1;
    if (cut && t1 < T && t1 - t0 > cut) t1 = t0 + ((t1 - t0) / cut) * cut;
    stages.push_back(t1);
    t0 = t1;
  }
  // images: one per input view (the x words carry that view's ranks)
  for (auto& rx : f->rx) {
    rx.top.assign(o[T] / 4, 0u);
    struct Item { int32_t v; uint32_t p; int l; };
    std::vector<Item> st;
    for (int t = 0; t < T; ++t) {
      const int64_t b = d->tree_offset[t];
      const uint32_t nt = ntop[t];
      uint32_t* top = &rx.top[o[t] / 4];
      uint2* bot = reinterpret_cast<uint2*>(top + 2 * NE);
      st.assign(1, Item{0, 1u, 0});
      while (!st.empty()) {
        const Item it = st.back();
        st.pop_back();
        const int64_t g = b + it.v;
        if (it.l == D0) {
          top[it.p] = (slot_of[g] - nt) * 8u;
          continue;
        }
        const bool leaf = d->feature[g] < 0;
        top[it.p] = leaf ? (rx.b8 ? kHxPad8 : kHxPad) : rx.recs[b + slot_of[g]].x;
        st.push_back(Item{leaf ? it.v : d->left[g], 2 * it.p, it.l + 1});
        st.push_back(Item{leaf ? it.v : d->right[g], 2 * it.p + 1, it.l + 1});
      }
      // a leaf that ends a path above depth D0 is entered through the top:
      // its bottom entries were set by the walk above (slot_of - nt)
      for (uint32_t v = nt; v < nt + nslots[t]; ++v) {
        uint2 r = rx.recs[b + v];
        if (v < f->h_rx_nint[t]) {
          const uint32_t lft = (r.y & 0xFFFFu) - nt, rgt = (r.y >> 16) - nt;
          r.y = ((rgt * 8u) << 16) | (lft * 8u);
        }
        bot[v - nt] = r;
      }
    }
  }
  f->h_lx_stage = stages;
  f->lx_stage_cap = static_cast<int64_t>(cap);
  const double per_stage = static_cast<double>(T) / static_cast<double>(stages.size() - 1);
  f->lx_ilp = cut ? cut : per_stage >= 7.5 ? 8 : per_stage >= 6.5 ? 7 : 4;
  f->hx_top = D0;
  f->layout = 9;
  return true;
}

// Layout 9 with a compact bottom (u8 bins only; treeinfer_kernels.h,
// t8explicit_predict_kernel).  A bottom node is one u32 -- the u8 record x
// word (bin offset | flags | rank << 16) with byte 3 holding a pair index
// k' -- and a node's children sit side by side at positions 2k', 2k' + 1, so
// a step reads the bin and the children's 8-byte pair at once (one LDS round
// trip, the bytes of layout 9's one record read) and selects the child.
// Positions: the entries (nodes at depth D0 and leaves above it, in the
// order the top reaches them) first, padded to an even count, then the
// children of the bottom's internal nodes in breadth-first order (internal
// node k's at n_entries + 2k), so k' = n_entries / 2 + k < 256 for trees of
// <= 255 leaves.  A leaf loops on itself: x = kLeaf | rank 0xFF (even
// position: never right, NaN-left) or rank 0 (odd: always right), bin offset
// 0, k' = p / 2; its value and ordinal are read by position from global
// tables when the group is walked.  Returns false (u8 layout 9 keeps its
// records) when a tree has more than 255 leaves or the images do not fit.
//
// The u16 form (b16, plan_tx16; t16explicit_predict_kernel) keeps the u16
// record x word's rank (high half), word index, half-word bit and NaN-left
// (low half, lane part cleared) and puts k' into bits 2-9 of the lane part;
// a leaf is rank 0xFFFF (even) / 0 (odd) with bin offset 0, and no internal
// node may have either rank (the leaf test).  It needs tiles of >= 256 rows
// (bits 2-9 inside the lane part).  Zero-missing forests lose the word's zero-flip
// bit: a 64-byte table of one bit per position sits between the top and the
// bottom (kT16ZfBytes), read only by the slow step.
bool plan_tx8(const ti_forest_desc* d, ti_forest* f, const std::vector<uint32_t>& slot_of, int D,
              bool b16 = false) {
  if (!b16 && (env_int("TI_TX8", 1) == 0 || !f->rx[0].b8 || !f->rx[1].b8)) return false;
  uint32_t bmask16 = 0, wmask16 = 0;
  if (b16) {
    if (env_int("TI_TX16", 1) == 0 || f->rx[0].b8 || f->rx[1].b8) return false;
    const int R = f->rx[0].rows;
    if (f->rx[1].rows != R || R < 256 || (R & (R - 1))) return false;
    int lg = 0;
    while ((1 << lg) < R) ++lg;
    wmask16 = (0xFFFFu << (2 + lg)) & 0xFFFFu;   // the word index bits
    bmask16 = wmask16 | 2u;
  }
  const uint32_t zfb = (b16 && f->zero_rule) ? ti::kT16ZfBytes : 0u;
  int D0 = env_int("TI_TX_TOP", b16 ? 8 : 6);
  // (the u16 bottom also runs without a top: D0 = 0, the root the only entry)
  D0 = std::max(b16 ? 0 : 1, std::min(D0, std::min(D, 10)));
  const int T = d->n_trees;
  const size_t NE = size_t(1) << D0;
  const uint32_t topb = static_cast<uint32_t>(8 * NE);
  const size_t acc_sz = f->accum == TI_F64 ? 8 : 4;
  // per tree: entries (the top's cut, left to right), then BFS children
  std::vector<std::vector<int32_t>> order(T);   // node at each bottom position (-1: pad)
  std::vector<std::vector<uint32_t>> kpair(T);  // per node: its children's pair index (internal)
  std::vector<uint32_t> pos(T + 1, 0), off(T + 1, 0);
  std::vector<int32_t> dep;
  struct Item { int32_t v; int l; };
  std::vector<Item> st;
  std::vector<int32_t> lvl, nxt;
  for (int t = 0; t < T; ++t) {
    const int64_t b = d->tree_offset[t];
    const int32_t n = static_cast<int32_t>(d->tree_offset[t + 1] - b);
    if (static_cast<int64_t>(n) > 509) return false;   // > 255 leaves
    std::vector<int32_t>& ord = order[t];
    ord.clear();
    // the top's cut in left-to-right order: depth-D0 nodes and shallow leaves
    st.assign(1, Item{0, 0});
    while (!st.empty()) {
      const Item it = st.back();
      st.pop_back();
      const int64_t g = b + it.v;
      if (it.l == D0 || d->feature[g] < 0) {
        ord.push_back(it.v);
        continue;
      }
      st.push_back(Item{d->right[g], it.l + 1});
      st.push_back(Item{d->left[g], it.l + 1});
    }
    const size_t n_entries = ord.size();
    if (n_entries & 1) ord.push_back(-1);
    const uint32_t half = static_cast<uint32_t>(ord.size() / 2);
    kpair[t].assign(n, 0u);
    uint32_t k = 0;
    // breadth-first over the bottom, a level at a time, each level's internal
    // nodes by cover (their children pairs: hot pairs first, cover_order)
    lvl.clear();
    for (const int32_t v : ord)
      if (v >= 0 && d->feature[b + v] >= 0) lvl.push_back(v);
    while (!lvl.empty()) {
      cover_order(d, b, &lvl);
      nxt.clear();
      for (const int32_t v : lvl) {
        if (half + k > 255) return false;
        kpair[t][v] = half + k++;
        for (const int32_t c : {d->left[b + v], d->right[b + v]}) {
          ord.push_back(c);
          if (d->feature[b + c] >= 0) nxt.push_back(c);
        }
      }
      lvl.swap(nxt);
    }
    pos[t + 1] = pos[t] + static_cast<uint32_t>(ord.size());
    const uint64_t bytes = topb + zfb + ((static_cast<uint64_t>(ord.size()) * 4 + 15) & ~uint64_t(15));
    if (bytes > 65520 || off[t] + bytes > 0xFFFFFFF0ull) return false;
    off[t + 1] = off[t] + static_cast<uint32_t>(bytes);
  }
  // stages: as plan_tx
  const int R = f->rx[0].rows;
  if (f->rx[1].rows != R) return false;
  const size_t bins = align16(static_cast<size_t>(std::max(f->rx[0].words, f->rx[1].words)) * R * 4 + 4);
  const int wgs = std::max(1, env_int("TI_LX_WGS", 2));
  size_t cap = kLdsPerCu / static_cast<size_t>(wgs);
  cap = cap > bins ? cap - bins : 0;
  cap = std::min(cap, static_cast<size_t>(kLxPf) * 16 * R) & ~size_t(15);
  size_t biggest = 0;
  for (int t = 0; t < T; ++t) biggest = std::max<size_t>(biggest, off[t + 1] - off[t]);
  if (T < 2 || cap < 2 * biggest) return false;
  // trees walked at once per lane: 4 (TI_LX_ILP overrides).  A stage holds a
  // whole number of ILP groups where it can (a group wider than the rest of
  // its stage walks duplicate trees): on c3_maxbin at 12 trees a stage, ILP 4
  // 4.70 ms, 7 5.29, 8 5.72 (profiles/r3_tx8_sweep.jsonl)
  const int force_ilp = env_int("TI_LX_ILP", 0);
  int ilp = force_ilp > 0 ? (force_ilp >= 8 ? 8 : force_ilp == 7 ? 7 : 4) : 4;
  // round 6: the u16 bottom two lanes a row when the tile's
  // 2R threads fit a workgroup of 512 and leaves are scalars (the lower lane
  // adds both halves' values in tree order); a group is 8 trees, 4 a lane.
  // TI_TX16_SPLIT=0 (developer knob) keeps the one-lane walk.
  const bool split = b16 && 2 * f->rx[0].rows <= 512 && d->leaf_width == 1 &&
                     env_int("TI_TX16_SPLIT", 1) != 0;
  if (b16) {   // the u16 kernel is instantiated at 4 and 8 trees a lane
    // (C3 at 1M rows, profiles/r5f_c3_t16_sweep.jsonl: 8 trees a lane and a
    // top of 8 levels 5.25-5.28 ms; 12 or 16 a lane 5.37-10.9 ms)
    ilp = split ? 8 : env_int("TI_TX16_ILP", 8) >= 8 ? 8 : 4;
  }
  std::vector<int32_t> stages(1, 0);
  int t0 = 0;
  while (t0 < T) {
    int t1 = t0 + 1;
    while (t1 < T && off[t1 + 1] - off[t0] <= cap) ++t1;
    if (t1 < T && t1 - t0 > ilp) {
      t1 = t0 + ((t1 - t0) / ilp) * ilp;
    }
    stages.push_back(t1);
    t0 = t1;
  }
  // position tables (shared by the views): leaf value and ordinal
  f->h_tx8_val.assign(static_cast<size_t>(pos[T]) * acc_sz, 0);
  f->h_tx8_ord.assign(pos[T], 0);
  for (int t = 0; t < T; ++t) {
    const int64_t b = d->tree_offset[t];
    for (uint32_t p = 0; p < pos[t + 1] - pos[t]; ++p) {
      const int32_t v = order[t][p];
      if (v < 0 || d->feature[b + v] >= 0) continue;
      const size_t at = pos[t] + p;
      f->h_tx8_ord[at] = static_cast<int32_t>(slot_of[b + v] - f->h_rx_nint[t]);
      if (acc_sz == 8) {
        const double x = d->leaf_value[(b + v) * d->leaf_width];
        std::memcpy(&f->h_tx8_val[at * 8], &x, 8);
      } else {
        const float x = static_cast<float>(d->leaf_value[(b + v) * d->leaf_width]);
        std::memcpy(&f->h_tx8_val[at * 4], &x, 4);
      }
    }
  }
  // images per view
  constexpr uint32_t kLeaf = ti::RxBins<true>::kLeaf, kNanLeft = ti::RxBins<true>::kNanLeft;
  std::vector<int32_t> entry_of;
  for (auto& rx : f->rx) {
    rx.top.assign(off[T] / 4, 0u);
    for (int t = 0; t < T; ++t) {
      const int64_t b = d->tree_offset[t];
      const int32_t n = static_cast<int32_t>(d->tree_offset[t + 1] - b);
      uint32_t* top = &rx.top[off[t] / 4];
      unsigned char* zf = reinterpret_cast<unsigned char*>(top + 2 * NE);
      uint32_t* bot = top + 2 * NE + zfb / 4;
      const std::vector<int32_t>& ord = order[t];
      entry_of.assign(n, -1);
      // a leaf word at position p: self-looping (even: rank 0xFF / 0xFFFF,
      // NaN-left; odd: rank 0), its own pair index
      auto leaf_word = [&](uint32_t p) {
        if (b16) return (p & 1 ? 0u : (0xFFFF0000u | 1u)) | ((p >> 1) << 2);
        return kLeaf | (p & 1 ? 0u : (0xFF0000u | kNanLeft)) | ((p >> 1) << 24);
      };
      for (uint32_t p = 0; p < ord.size(); ++p) {
        const int32_t v = ord[p];
        if (v < 0) {
          bot[p] = leaf_word(p);
          continue;
        }
        if (entry_of[v] < 0) entry_of[v] = static_cast<int32_t>(p);
        const int64_t g = b + v;
        if (d->feature[g] < 0) {
          bot[p] = leaf_word(p);
        } else if (b16) {
          const uint32_t xw = rx.recs[b + slot_of[g]].x;
          const uint32_t rk = xw >> 16;
          if (rk == 0u || rk == 0xFFFFu) return false;   // the ranks that mark a leaf
          bot[p] = (xw & (0xFFFF0000u | wmask16 | 3u)) | (kpair[t][v] << 2);
          if (zfb && (xw & ti::kRxZeroFlip)) zf[p >> 3] |= static_cast<unsigned char>(1u << (p & 7));
        } else {
          bot[p] = rx.recs[b + slot_of[g]].x | (kpair[t][v] << 24);
        }
      }
      // the top: x words, and at depth D0 the entry position
      struct TItem { int32_t v; uint32_t hp; int l; };
      std::vector<TItem> ts(1, TItem{0, 1u, 0});
      while (!ts.empty()) {
        const TItem it = ts.back();
        ts.pop_back();
        const int64_t g = b + it.v;
        if (it.l == D0) {
          top[it.hp] = static_cast<uint32_t>(entry_of[it.v]);
          continue;
        }
        const bool leaf = d->feature[g] < 0;
        top[it.hp] = leaf ? (b16 ? kHxPad : kHxPad8) : rx.recs[b + slot_of[g]].x;
        ts.push_back(TItem{leaf ? it.v : d->left[g], 2 * it.hp, it.l + 1});
        ts.push_back(TItem{leaf ? it.v : d->right[g], 2 * it.hp + 1, it.l + 1});
      }
    }
  }
  f->h_tx_off = off;
  f->h_tx8_pos = pos;
  f->h_tx_nint.assign(T, 0);
  f->h_lx_stage = stages;
  f->lx_stage_cap = static_cast<int64_t>(cap);
  f->lx_ilp = ilp;
  f->hx_top = D0;
  f->tx8 = split ? 3 : b16 ? 2 : 1;
  f->tx16_mask = bmask16;
  f->layout = 9;
  return true;
}

// Mean depth of the leaves of a forest (every leaf counted once).
double mean_leaf_depth(const ti_forest_desc* d) {
  double sum = 0;
  int64_t n_leaf = 0;
  std::vector<int32_t> dep, q;
  for (int t = 0; t < d->n_trees; ++t) {
    const int64_t b = d->tree_offset[t];
    const int32_t n = static_cast<int32_t>(d->tree_offset[t + 1] - b);
    dep.assign(n, 0);
    q.assign(1, 0);   // breadth-first: a parent's depth is set first
    for (size_t qi = 0; qi < q.size(); ++qi) {
      const int32_t v = q[qi];
      const int64_t g = b + v;
      if (d->feature[g] < 0) {
        sum += dep[v];
        ++n_leaf;
      } else {
        dep[d->left[g]] = dep[d->right[g]] = dep[v] + 1;
        q.push_back(d->left[g]);
        q.push_back(d->right[g]);
      }
    }
  }
  return n_leaf ? sum / n_leaf : 0.0;
}

// TreeSHAP path tables + bias (see ShapPath).  Forests without covers or
// with categorical splits get none (TI_OUTPUT_CONTRIB is then unsupported).
struct ShapBuilder {
  const ti_forest_desc* d;
  ti_forest* f;
  int64_t b = 0;
  int group = 0;
  std::vector<ShapElem> cur;

  void dfs(int32_t v) {
    const int64_t g = b + v;
    const int LW = d->leaf_width;
    if (d->feature[g] < 0) {
      ShapPath p;
      p.group = group;
      p.n = static_cast<int32_t>(cur.size());
      p.first = static_cast<int64_t>(f->h_elems.size());
      p.leaf = static_cast<int64_t>(f->h_path_leaf.size()) / LW;
      f->h_elems.insert(f->h_elems.end(), cur.begin(), cur.end());
      for (int k = 0; k < LW; ++k) f->h_path_leaf.push_back(d->leaf_value[g * LW + k]);
      f->h_paths.push_back(p);
      f->shap_maxl = std::max(f->shap_maxl, p.n);
      return;
    }
    const int32_t fe = d->feature[g];
    const double t = d->threshold[g];
    const bool nan_left = (d->flags[g] & TI_NODE_NAN_LEFT) != 0;
    const bool zero_left = (d->flags[g] & TI_NODE_ZERO_FLIP) ? !(0 <= t) : (0 <= t);
    for (int side = 0; side < 2; ++side) {
      const bool left = side == 0;
      const int32_t child = left ? d->left[g] : d->right[g];
      const std::vector<ShapElem> saved = cur;
      ShapElem e{fe, kShapNanOk | kShapZeroOk, -INFINITY, INFINITY, 1.0};
      for (size_t i = 0; i < cur.size(); ++i)
        if (cur[i].feature == fe) {   // unwind the earlier split on fe, re-extend at the end
          e = cur[i];
          cur.erase(cur.begin() + static_cast<std::ptrdiff_t>(i));
          break;
        }
      e.zf = (d->cover[b + child] / d->cover[g]) * e.zf;
      if (left) {
        if (std::isnan(t)) e.flags |= kShapEmpty;
        else e.hi = std::min(e.hi, t);
      } else if (!std::isnan(t)) {
        e.lo = std::max(e.lo, t);
      }
      if (nan_left != left) e.flags &= ~kShapNanOk;
      if (zero_left != left) e.flags &= ~kShapZeroOk;
      cur.push_back(e);
      dfs(child);
      cur = saved;
    }
  }

  std::vector<double> mean(int32_t v) {   // FillNodeMeanValues, per leaf-vector entry
    const int64_t g = b + v;
    const int LW = d->leaf_width;
    std::vector<double> r(LW);
    if (d->feature[g] < 0) {
      for (int k = 0; k < LW; ++k) r[k] = d->leaf_value[g * LW + k];
      return r;
    }
    const int32_t l = d->left[g], rr = d->right[g];
    const std::vector<double> ml = mean(l), mr = mean(rr);
    for (int k = 0; k < LW; ++k)
      r[k] = (ml[k] * d->cover[b + l] + mr[k] * d->cover[b + rr]) / d->cover[g];
    return r;
  }
};

// At create: whether contributions are possible (covers, no categorical
// splits), and the host copy build_shap will read on first use.
void keep_shap_source(const ti_forest_desc* d, ti_forest* f) {
  if (!d->cover) return;
  for (int64_t g = 0; g < d->n_nodes; ++g)
    if (d->feature[g] >= 0 && (d->flags[g] & TI_NODE_CATEGORICAL)) return;
  auto src = std::make_unique<ti_forest::ShapSource>();
  const int64_t N = d->n_nodes, T = d->n_trees;
  src->tree_offset.assign(d->tree_offset, d->tree_offset + T + 1);
  if (d->tree_group) src->tree_group.assign(d->tree_group, d->tree_group + T);
  src->feature.assign(d->feature, d->feature + N);
  src->left.assign(d->left, d->left + N);
  src->right.assign(d->right, d->right + N);
  src->threshold.assign(d->threshold, d->threshold + N);
  src->leaf_value.assign(d->leaf_value, d->leaf_value + N * d->leaf_width);
  src->base_margin.assign(d->base_margin, d->base_margin + d->n_groups);
  src->cover.assign(d->cover, d->cover + N);
  src->flags.assign(d->flags, d->flags + N);
  src->desc = *d;
  src->desc.tree_offset = src->tree_offset.data();
  src->desc.tree_group = src->tree_group.empty() ? nullptr : src->tree_group.data();
  src->desc.feature = src->feature.data();
  src->desc.left = src->left.data();
  src->desc.right = src->right.data();
  src->desc.threshold = src->threshold.data();
  src->desc.leaf_value = src->leaf_value.data();
  src->desc.base_margin = src->base_margin.data();
  src->desc.cover = src->cover.data();
  src->desc.flags = src->flags.data();
  src->desc.leaf_id = nullptr;
  src->desc.cat_bits = nullptr;
  src->desc.cat_offset = nullptr;
  src->desc.cat_nwords = nullptr;
  f->shap_src = std::move(src);
  f->has_shap = 1;
}

void build_shap(const ti_forest_desc* d, ti_forest* f) {
  const int K = d->n_groups;
  std::vector<double> bias(K);
  for (int k = 0; k < K; ++k) bias[k] = d->base_margin[k] * d->average_divisor;
  ShapBuilder sb{d, f};
  for (int t = 0; t < d->n_trees; ++t) {
    sb.b = d->tree_offset[t];
    sb.group = d->leaf_width == 1 ? d->tree_group[t] : 0;
    sb.cur.clear();
    sb.dfs(0);
    const std::vector<double> m = sb.mean(0);
    if (d->leaf_width == 1) bias[sb.group] += m[0];
    else for (int k = 0; k < K; ++k) bias[k] += m[k];
  }
  f->h_shap_bias.resize(K);
  for (int k = 0; k < K; ++k) f->h_shap_bias[k] = bias[k] / d->average_divisor;
  f->shap_npaths = static_cast<int64_t>(f->h_paths.size());
}

int upload_device(ti_forest* f, DeviceForest& d, int device) {
  d.device = device;
  TI_HIP(hipSetDevice(device));
  TI_HIP(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
  int rc;
  if ((rc = upload(&d.tree_group, f->h_group, &d.bytes))) return rc;
  if (f->layout == 0) {
    if ((rc = upload(&d.heap32, f->h_heap32, &d.bytes))) return rc;
    if ((rc = upload(&d.heap64, f->h_heap64, &d.bytes))) return rc;
    if ((rc = upload(&d.heap_leaf_ids, f->h_heap_leaf_ids, &d.bytes))) return rc;
  } else if (f->layout == 6 || f->layout == 7 || f->layout == 8) {
    for (int i = 0; i < 2; ++i) {
      if ((rc = upload(&d.rx_recs[i], f->rx[i].recs, &d.bytes))) return rc;
      if ((rc = upload(&d.bx_tbl[i], f->rx[i].tbl, &d.bytes))) return rc;
      if (f->layout == 8 && (rc = upload(&d.hx_top[i], f->rx[i].top, &d.bytes))) return rc;
    }
    if ((rc = upload(&d.rx_base, f->h_rx_base, &d.bytes))) return rc;
    if ((rc = upload(&d.rx_nint, f->h_rx_nint, &d.bytes))) return rc;
    if (f->layout == 7 && (rc = upload(&d.lx_stage, f->h_lx_stage, &d.bytes))) return rc;
    if ((rc = upload(&d.leaf_base, f->h_leaf_base, &d.bytes))) return rc;
    if (f->LW > 1) {   // vector leaves are read from the leaf table
      unsigned char* lv = nullptr;
      if ((rc = upload(&lv, f->h_leaves, &d.bytes))) return rc;
      d.leaves = lv;
    }
    if ((rc = upload(&d.exp_leaf_ids, f->h_exp_leaf_ids, &d.bytes))) return rc;
  } else if (f->layout == 9) {
    for (int i = 0; i < 2; ++i) {
      if ((rc = upload(&d.hx_top[i], f->rx[i].top, &d.bytes))) return rc;
      if ((rc = upload(&d.bx_tbl[i], f->rx[i].tbl, &d.bytes))) return rc;
    }
    if ((rc = upload(&d.rx_base, f->h_tx_off, &d.bytes))) return rc;
    if ((rc = upload(&d.rx_nint, f->h_tx_nint, &d.bytes))) return rc;
    if (f->tx8) {
      if ((rc = upload(&d.tx8_pos, f->h_tx8_pos, &d.bytes))) return rc;
      unsigned char* tv = nullptr;
      if ((rc = upload(&tv, f->h_tx8_val, &d.bytes))) return rc;
      d.tx8_val = tv;
      if ((rc = upload(&d.tx8_ord, f->h_tx8_ord, &d.bytes))) return rc;
    }
    if ((rc = upload(&d.lx_stage, f->h_lx_stage, &d.bytes))) return rc;
    if ((rc = upload(&d.leaf_base, f->h_leaf_base, &d.bytes))) return rc;
    if (f->LW > 1) {   // vector leaves are read from the leaf table
      unsigned char* lv = nullptr;
      if ((rc = upload(&lv, f->h_leaves, &d.bytes))) return rc;
      d.leaves = lv;
    }
    if ((rc = upload(&d.exp_leaf_ids, f->h_exp_leaf_ids, &d.bytes))) return rc;
  } else if (f->layout == 3) {
    for (int i = 0; i < 2; ++i) {
      if ((rc = upload(&d.bh_img[i], f->bh[i].img, &d.bytes))) return rc;
      if ((rc = upload(&d.bh_tbl[i], f->bh[i].tbl, &d.bytes))) return rc;
    }
    // the permuted image of the fixed walk (float32 view only): once per replica
    if ((rc = upload(&d.bh_fix_img, f->bh[0].fix_img, &d.bytes))) return rc;
    if ((rc = upload(&d.heap_leaf_ids, f->h_heap_leaf_ids, &d.bytes))) return rc;
  } else {
    if ((rc = upload(&d.nodes, f->h_nodes, &d.bytes))) return rc;
    if ((rc = upload(&d.thr64, f->h_thr64, &d.bytes))) return rc;
    if ((rc = upload(&d.node_base, f->h_node_base, &d.bytes))) return rc;
    if ((rc = upload(&d.root, f->h_root, &d.bytes))) return rc;
    if ((rc = upload(&d.leaf_base, f->h_leaf_base, &d.bytes))) return rc;
    unsigned char* lv = nullptr;
    if ((rc = upload(&lv, f->h_leaves, &d.bytes))) return rc;
    d.leaves = lv;
    if ((rc = upload(&d.exp_leaf_ids, f->h_exp_leaf_ids, &d.bytes))) return rc;
    if ((rc = upload(&d.cat_words, f->h_cat_words, &d.bytes))) return rc;
  }
  return TI_OK;
}

// ----------------------------------------------------------------- launch
using ti::KernelFn;

// Kernel instantiations live in one translation unit per (input, accumulator)
// type pair (treeinfer_k_*.hip, compiled in parallel); see treeinfer_dispatch.h.
KernelFn select_kernel(int layout, int xdt, int accum, int K, bool fl, bool z) {
  if (xdt == TI_F32 && accum == TI_F32) return ti::kernels_ff(layout, K, fl, z, false, 0);
  if (xdt == TI_F32 && accum == TI_F64) return ti::kernels_fd(layout, K, fl, z, false, 0);
  if (xdt == TI_F64 && accum == TI_F64) return ti::kernels_dd(layout, K, fl, z, false, 0);
  return ti::kernels_df(layout, K, fl, z, false, 0);
}

KernelFn select_bheap(int xdt, int accum, int K, bool b16, int pf) {
  if (xdt == TI_F32 && accum == TI_F32) return ti::kernels_ff(3, K, true, false, b16, pf);
  if (xdt == TI_F32 && accum == TI_F64) return ti::kernels_fd(3, K, true, false, b16, pf);
  if (xdt == TI_F64 && accum == TI_F64) return ti::kernels_dd(3, K, true, false, b16, pf);
  return ti::kernels_df(3, K, true, false, b16, pf);
}

KernelFn select_rexplicit(int xdt, int accum, int K, bool z, int ilp) {
  if (xdt == TI_F32 && accum == TI_F32) return ti::kernels_ff(6, K, true, z, true, ilp);
  if (xdt == TI_F32 && accum == TI_F64) return ti::kernels_fd(6, K, true, z, true, ilp);
  if (xdt == TI_F64 && accum == TI_F64) return ti::kernels_dd(6, K, true, z, true, ilp);
  return ti::kernels_df(6, K, true, z, true, ilp);
}

KernelFn select_lexplicit(int xdt, int accum, int K, bool z, int ilp) {
  if (xdt == TI_F32 && accum == TI_F32) return ti::kernels_ff(7, K, true, z, true, ilp);
  if (xdt == TI_F32 && accum == TI_F64) return ti::kernels_fd(7, K, true, z, true, ilp);
  if (xdt == TI_F64 && accum == TI_F64) return ti::kernels_dd(7, K, true, z, true, ilp);
  return ti::kernels_df(7, K, true, z, true, ilp);
}

// Columns per pass of the record layouts' coalesced binning through the stage
// area (rx_stage_bins): a multiple of 8 that fits `bytes` for R rows, at most
// the features rounded up to 8; 0 (per-lane row loads) when fewer than 8 fit.
int32_t bin_chunk_for(size_t bytes, int R, int xdt, int F) {
  const size_t per_col = static_cast<size_t>(R) * (xdt == TI_F64 ? 8 : 4);
  size_t c = (bytes / per_col) & ~size_t(7);
  c = std::min(c, static_cast<size_t>((F + 7) & ~7));
  return c >= 8 ? static_cast<int32_t>(c) : 0;
}

KernelFn select_texplicit(int xdt, int accum, int K, bool z, int ilp, bool b8) {
  if (xdt == TI_F32 && accum == TI_F32) return ti::kernels_ff(9, K, true, z, !b8, ilp);
  if (xdt == TI_F32 && accum == TI_F64) return ti::kernels_fd(9, K, true, z, !b8, ilp);
  if (xdt == TI_F64 && accum == TI_F64) return ti::kernels_dd(9, K, true, z, !b8, ilp);
  return ti::kernels_df(9, K, true, z, !b8, ilp);
}

KernelFn select_t8explicit(int xdt, int accum, int K, bool z, int ilp) {   // layout 9, compact u8 bottom
  if (xdt == TI_F32 && accum == TI_F32) return ti::kernels_ff(11, K, true, z, false, ilp);
  if (xdt == TI_F32 && accum == TI_F64) return ti::kernels_fd(11, K, true, z, false, ilp);
  if (xdt == TI_F64 && accum == TI_F64) return ti::kernels_dd(11, K, true, z, false, ilp);
  return ti::kernels_df(11, K, true, z, false, ilp);
}

KernelFn select_t16explicit(int xdt, int accum, int K, bool z, int ilp) {   // layout 9, compact u16 bottom
  if (xdt == TI_F32 && accum == TI_F32) return ti::kernels_ff(12, K, true, z, true, ilp);
  if (xdt == TI_F32 && accum == TI_F64) return ti::kernels_fd(12, K, true, z, true, ilp);
  if (xdt == TI_F64 && accum == TI_F64) return ti::kernels_dd(12, K, true, z, true, ilp);
  return ti::kernels_df(12, K, true, z, true, ilp);
}

KernelFn select_t16split(int xdt, int accum, int K, bool z) {   // layout 9, u16, two lanes a row
  if (xdt == TI_F32 && accum == TI_F32) return ti::kernels_ff(13, K, true, z, true, 4);
  if (xdt == TI_F32 && accum == TI_F64) return ti::kernels_fd(13, K, true, z, true, 4);
  if (xdt == TI_F64 && accum == TI_F64) return ti::kernels_dd(13, K, true, z, true, 4);
  return ti::kernels_df(13, K, true, z, true, 4);
}

KernelFn select_hexplicit(int xdt, int accum, int K, bool z, int ilp) {
  if (xdt == TI_F32 && accum == TI_F32) return ti::kernels_ff(8, K, true, z, true, ilp);
  if (xdt == TI_F32 && accum == TI_F64) return ti::kernels_fd(8, K, true, z, true, ilp);
  if (xdt == TI_F64 && accum == TI_F64) return ti::kernels_dd(8, K, true, z, true, ilp);
  return ti::kernels_df(8, K, true, z, true, ilp);
}

std::mutex g_attr_mu;
std::set<std::pair<int, const void*>> g_attr_done;

// Once per (device, kernel): the kernels address LDS as offsets from 0, which
// holds only while they declare no static LDS -- check it, then raise the
// dynamic-LDS limit to the whole 160 KiB.
int ensure_lds_attr(int device, KernelFn fn) {
  std::lock_guard<std::mutex> lk(g_attr_mu);
  auto key = std::make_pair(device, reinterpret_cast<const void*>(fn));
  if (g_attr_done.count(key)) return TI_OK;
  hipFuncAttributes attr;
  TI_HIP(hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(fn)));
  if (attr.sharedSizeBytes != 0)
    return fail(TI_ERR_DEVICE, "kernel declares " + std::to_string(attr.sharedSizeBytes) +
                                   " B of static LDS; the LDS-address-0 layout is violated");
  TI_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                             hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kLdsPerCu)));
  g_attr_done.insert(key);
  return TI_OK;
}

// TI_OCC=1: print, once per kernel, the workgroups per CU the runtime's
// occupancy calculator allows for this launch shape (a diagnostic for the
// PMC passes' resident-wave counts).
void occ_note(KernelFn fn, int block, size_t lds) {
  static const int on = env_int("TI_OCC", 0);
  if (!on) return;
  static std::mutex mu;
  static std::set<const void*> seen;
  std::lock_guard<std::mutex> lk(mu);
  if (!seen.insert(reinterpret_cast<const void*>(fn)).second) return;
  int n = -1;
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(fn), block, lds);
  hipFuncAttributes attr;
  (void)hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(fn));
  std::fprintf(stderr, "[ti occupancy] block %d lds %zu B: %d workgroups/CU (%d waves/SIMD), %d VGPRs, %d SGPRs\n",
               block, lds, n, n * ((block + 63) / 64) / 4, attr.numRegs, 0);
}

int64_t output_width(const ti_forest* f, int kind) {
  if (kind == TI_OUTPUT_LEAF) return f->T;
  if (kind == TI_OUTPUT_CONTRIB) return static_cast<int64_t>(f->K) * (f->F + 1);
  if (kind == TI_OUTPUT_PREDICT && f->transform == TI_TRANSFORM_ARGMAX) return 1;
  return f->K;
}

int output_dtype(const ti_forest* f, int kind) {
  if (kind == TI_OUTPUT_LEAF) return TI_I32;
  return f->accum;
}

size_t dtype_size(int dt) { return dt == TI_F64 ? 8 : 4; }

// Whether a binned-heap launch takes the fixed-layout walk (bheap_fix_kernel):
// float32 input and sums, one scalar leaf per leaf, depth-8 records of 2 KB,
// 512-row tiles (the node words carry their heap index) and at most 14 bin
// words (the image ends below kFixFlag); leaf ids keep the indexed walk.
// TI_BHEAP_FIX=0 turns it off.
bool bheap_fixed(const ti_forest* f, int xdt, int kind) {
  if (f->layout != 3 || xdt != TI_F32 || f->accum != TI_F32 || f->LW != 1 || f->depth != 8)
    return false;
  if (kind != TI_OUTPUT_MARGIN && kind != TI_OUTPUT_PREDICT) return false;
  const ti_forest::BinImage& bi = f->bh[0];
  return env_int("TI_BHEAP_FIX", 1) != 0 && bi.rows == ti::kFixRows && bi.mask == ti::kBNodeOffMask512 &&
         bi.stride == ti::kFixTree && static_cast<uint32_t>(bi.words) * 2048u <= ti::kFixFlag;
}

int launch(ti_forest* f, DeviceForest& d, const void* X, int xdt, int64_t rows, int32_t cols,
           int64_t stride, int kind, void* out, hipStream_t stream) {
  if (rows <= 0) return TI_OK;
  const size_t xs = dtype_size(xdt);
  // rows per tile = threads per workgroup; the heap images fixed it at create
  // time (their meta words hold [F][R] byte offsets)
  int R;
  if (f->layout == 0) {
    R = xdt == TI_F64 ? f->rows64 : f->rows32;
  } else if (f->layout == 3) {
    R = f->bh[xdt == TI_F64 ? 1 : 0].rows;
  } else if (f->layout >= 6 && f->layout <= 9) {
    R = f->rx[xdt == TI_F64 ? 1 : 0].rows;
  } else {
    R = 256;
    while (R > 64 && static_cast<size_t>(f->F) * R * xs > kFeatLdsMax) R >>= 1;
    if (static_cast<size_t>(f->F) * R * xs > kFeatLdsMax) R = 0;
  }
  const bool feat_lds = R > 0;
  if (!feat_lds) R = 256;
  size_t feat_bytes = feat_lds ? align16(static_cast<size_t>(f->F) * R * xs) : 0;
  if (f->layout == 3) feat_bytes = static_cast<size_t>(f->bh[xdt == TI_F64 ? 1 : 0].words) * R * 4;
  if (f->layout >= 6 && f->layout <= 9)
    feat_bytes = static_cast<size_t>(f->rx[xdt == TI_F64 ? 1 : 0].words) * R * 4;

  KArgs a;
  std::memset(&a, 0, sizeof(a));
  a.X = X;
  a.n_rows = rows;
  a.row_stride = stride;
  a.n_cols = cols;
  a.n_features = f->F;
  a.n_trees = f->T;
  a.n_groups = f->K;
  a.leaf_width = f->LW;
  a.kind = kind;
  a.transform = f->transform;
  a.base_first = f->base_first;
  a.lgb_zero_map = f->lgb_zero_map;
  a.divide = f->divisor != 1.0;
  a.transform_param = f->tparam;
  a.average_divisor = f->divisor;
  for (int k = 0; k < ti::kMaxGroups; ++k) a.base[k] = f->base[k];
  a.tree_group = d.tree_group;
  a.out = out;

  size_t lds = feat_bytes + 16;
  if (f->layout == 0) {
    const int64_t stride_b = xdt == TI_F64 ? f->stride64 : f->stride32;
    a.trees = xdt == TI_F64 ? d.heap64 : d.heap32;
    a.tree_stride = stride_b;
    a.heap_leaf_ids = d.heap_leaf_ids;
    a.depth = f->depth;
    // Stage size S (trees): as many trees as keep the workgroups-per-CU count
    // that the smallest useful stage (kTilp trees) allows -- occupancy is what
    // hides the LDS latency of the walk (measured: 3 WG/CU beat 2 WG/CU by
    // 1.7x at F = 28) -- capped by the prefetch registers (kPf x 16 B x R).
    // TI_HEAP_LDS_KB overrides with a fixed per-workgroup budget.
    const size_t fixed = feat_bytes + 16;   // feature image + NaN flag word
    const int64_t cap = static_cast<int64_t>(ti::kPf) * 16 * R / stride_b;
    auto wgs = [&](int64_t n) { return kLdsPerCu / (fixed + static_cast<size_t>(n * stride_b)); };
    static const int budget_kb = env_int("TI_HEAP_LDS_KB", 0);
    int64_t S;
    if (budget_kb > 0) {
      const size_t b = static_cast<size_t>(budget_kb) * 1024;
      S = b > fixed ? static_cast<int64_t>((b - fixed) / stride_b) : 0;
      if (S >= ti::kTilp) S -= S % ti::kTilp;
    } else {
      S = std::min<int64_t>(ti::kTilp, cap);
      while (S > 1 && fixed + static_cast<size_t>(S * stride_b) > kLdsPerCu) --S;
      const size_t best = S >= 1 ? wgs(S) : 0;
      while (S + ti::kTilp <= cap && S + ti::kTilp <= f->T && wgs(S + ti::kTilp) >= best)
        S += ti::kTilp;
    }
    if (S < 1 || fixed + static_cast<size_t>(S * stride_b) > kLdsPerCu)
      return fail(TI_ERR_UNSUPPORTED, "heap tree record does not fit in LDS");
    S = std::min<int64_t>(S, cap);
    S = std::min<int64_t>(S, f->T);
    a.stage_trees = static_cast<int32_t>(S);
    lds = fixed + static_cast<size_t>(S * stride_b);
  } else if (f->layout == 3) {
    // binned heap: [bin image][flag][stage area = S tree records, also the
    // binning temp of >= 8 columns].  S as for the heap layout: the most
    // trees that keep the best workgroups-per-CU count, capped by the
    // prefetch registers (PF x 16 B x R).
    const int ii = xdt == TI_F64 ? 1 : 0;
    const ti_forest::BinImage& bi = f->bh[ii];
    const int64_t stride_b = bi.stride;
    const size_t fixed = align16(feat_bytes + 4);
    const size_t temp_min = 8 * static_cast<size_t>(R) * xs;
    auto area = [&](int64_t n) { return std::max(static_cast<size_t>(n * stride_b), temp_min); };
    auto wgs = [&](int64_t n) { return kLdsPerCu / (fixed + area(n)); };
    const int64_t cap = static_cast<int64_t>(8) * 16 * R / stride_b;
    int64_t S = std::min<int64_t>(ti::kBTilp, cap);
    if (S < 1) return fail(TI_ERR_UNSUPPORTED, "binned heap tree record does not fit the stage");
    const size_t best = wgs(S);
    while (S + ti::kBTilp <= cap && S + ti::kBTilp <= f->T && wgs(S + ti::kBTilp) >= best) S += ti::kBTilp;
    static const int force_s = env_int("TI_BHEAP_STAGE", 0);
    if (force_s > 0) S = std::min<int64_t>(force_s, cap);
    S = std::min<int64_t>(S, f->T);
    const int pf = S * stride_b <= static_cast<int64_t>(4) * 16 * R ? 4 : 8;
    a.X = X;
    a.bin_mask = bi.mask;
    a.bin_kary = bi.kary;
    a.trees = d.bh_img[ii];
    a.tree_stride = stride_b;
    a.heap_leaf_ids = d.heap_leaf_ids;
    const bool fix_perm = d.bh_fix_img != nullptr && bheap_fixed(f, xdt, kind);
    a.depth = f->depth;
    a.stage_trees = static_cast<int32_t>(S);
    a.bin_tbl = d.bh_tbl[ii];
    a.bin_L = bi.L;
    a.bin_words = bi.words;
    a.stage_off = static_cast<int32_t>(fixed);
    const size_t ar = area(S);
    a.bin_chunk = static_cast<int32_t>(std::min<size_t>((ar / (static_cast<size_t>(R) * xs)) & ~size_t(7),
                                                        static_cast<size_t>(f->F + 7) & ~size_t(7)));
    lds = fixed + ar;
    KernelFn fn = select_bheap(xdt, f->accum, f->K, bi.b16 != 0, pf);
    if (bheap_fixed(f, xdt, kind)) {
      // fixed layout (bheap_fix_kernel): [bins][flag][NG groups of 4 trees at
      // kFixStage]; the binning goes through the stage area, 4 NG columns at a
      // time.  NG = 1: 38,912 B, 4 workgroups (32 waves) per CU
      const int ng = std::min(2, std::max(1, env_int("TI_BHEAP_NG", 1)));
      fn = ti::kernels_ff(10, f->K, true, false, bi.b16 != 0, ng);
      a.stage_trees = 4 * ng;
      a.bin_chunk = 4 * ng;
      a.stage_off = static_cast<int32_t>(ti::kFixStage);
      if (fix_perm) a.trees = d.bh_fix_img;   // same walk, hot pair slots first
      lds = ti::kFixStage + static_cast<size_t>(4 * ng) * ti::kFixTree;
    }
    int rc = ensure_lds_attr(d.device, fn);
    if (rc) return rc;
    const int64_t grid = (rows + R - 1) / R;
    if (grid > 0x7fffffff) return fail(TI_ERR_INVALID, "too many rows for one launch");
    occ_note(fn, R, lds);
  hipLaunchKernelGGL(fn, dim3(static_cast<unsigned>(grid)), dim3(R), lds, stream, a);
    TI_HIP(hipGetLastError());
    return TI_OK;
  } else if (f->layout == 6) {
    const int ii = xdt == TI_F64 ? 1 : 0;
    const ti_forest::RecExplicit& rx = f->rx[ii];
    a.rx_recs = d.rx_recs[ii];
    a.rx_base = d.rx_base;
    a.rx_nint = d.rx_nint;
    a.leaf_base = d.leaf_base;
    a.rx_slots = static_cast<uint32_t>(f->rx_slots);
    a.leaves = d.leaves;
    a.exp_leaf_ids = d.exp_leaf_ids;
    a.bin_tbl = d.bx_tbl[ii];
    a.bin_L = rx.L;
    a.bin_kary = rx.kary;
    a.bin_words = rx.words;
    lds = feat_bytes + 16;
    KernelFn fn = select_rexplicit(xdt, f->accum, f->K, f->zero_rule != 0, f->rx_ilp);
    int rc = ensure_lds_attr(d.device, fn);
    if (rc) return rc;
    const int64_t grid = (rows + R - 1) / R;
    if (grid > 0x7fffffff) return fail(TI_ERR_INVALID, "too many rows for one launch");
    occ_note(fn, R, lds);
  hipLaunchKernelGGL(fn, dim3(static_cast<unsigned>(grid)), dim3(R), lds, stream, a);
    TI_HIP(hipGetLastError());
    return TI_OK;
  } else if (f->layout == 7) {
    const int ii = xdt == TI_F64 ? 1 : 0;
    const ti_forest::RecExplicit& rx = f->rx[ii];
    a.rx_recs = d.rx_recs[ii];
    a.rx_base = d.rx_base;
    a.rx_nint = d.rx_nint;
    a.leaf_base = d.leaf_base;
    a.rx_slots = static_cast<uint32_t>(f->rx_slots);
    a.leaves = d.leaves;
    a.exp_leaf_ids = d.exp_leaf_ids;
    a.bin_tbl = d.bx_tbl[ii];
    a.bin_L = rx.L;
    a.bin_kary = rx.kary;
    a.bin_words = rx.words;
    a.stage_start = d.lx_stage;
    a.n_stages = static_cast<int32_t>(f->h_lx_stage.size() - 1);
    a.stage_off = static_cast<int32_t>(align16(feat_bytes + 4));
    lds = std::max(static_cast<size_t>(a.stage_off) + static_cast<size_t>(f->lx_stage_cap), kLxMinLds);
    if (lds > kLdsPerCu || static_cast<int64_t>(kLxPf) * 16 * R < f->lx_stage_cap)
      return fail(TI_ERR_UNSUPPORTED, "staged record layout exceeds LDS");
    a.bin_chunk = bin_chunk_for(static_cast<size_t>(f->lx_stage_cap), R, xdt, f->F);
    KernelFn fn = select_lexplicit(xdt, f->accum, f->K, f->zero_rule != 0, f->lx_ilp);
    int rc = ensure_lds_attr(d.device, fn);
    if (rc) return rc;
    const int64_t grid = (rows + R - 1) / R;
    if (grid > 0x7fffffff) return fail(TI_ERR_INVALID, "too many rows for one launch");
    occ_note(fn, R, lds);
  hipLaunchKernelGGL(fn, dim3(static_cast<unsigned>(grid)), dim3(R), lds, stream, a);
    TI_HIP(hipGetLastError());
    return TI_OK;
  } else if (f->layout == 9) {
    const int ii = xdt == TI_F64 ? 1 : 0;
    const ti_forest::RecExplicit& rx = f->rx[ii];
    a.trees = reinterpret_cast<const unsigned char*>(d.hx_top[ii]);
    a.depth = f->hx_top;
    a.rx_base = d.rx_base;   // tree byte offsets in the image
    a.rx_nint = d.rx_nint;   // bottom internal nodes
    a.leaf_base = d.leaf_base;
    a.leaves = d.leaves;
    a.exp_leaf_ids = d.exp_leaf_ids;
    a.bin_tbl = d.bx_tbl[ii];
    a.bin_L = rx.L;
    a.bin_kary = rx.kary;
    a.bin_words = rx.words;
    a.stage_start = d.lx_stage;
    a.n_stages = static_cast<int32_t>(f->h_lx_stage.size() - 1);
    a.stage_off = static_cast<int32_t>(align16(feat_bytes + 4));
    lds = std::max(static_cast<size_t>(a.stage_off) + static_cast<size_t>(f->lx_stage_cap), kLxMinLds);
    if (lds > kLdsPerCu || static_cast<int64_t>(kLxPf) * 16 * R < f->lx_stage_cap)
      return fail(TI_ERR_UNSUPPORTED, "heap-top staged layout exceeds LDS");
    a.bin_chunk = bin_chunk_for(static_cast<size_t>(f->lx_stage_cap), R, xdt, f->F);
    a.tx_pos = d.tx8_pos;
    a.tx_vals = d.tx8_val;
    a.tx_ord = d.tx8_ord;
    a.bin_mask = f->tx16_mask;
    KernelFn fn = f->tx8 == 3 ? select_t16split(xdt, f->accum, f->K, f->zero_rule != 0)
                : f->tx8 == 2 ? select_t16explicit(xdt, f->accum, f->K, f->zero_rule != 0, f->lx_ilp)
                : f->tx8 ? select_t8explicit(xdt, f->accum, f->K, f->zero_rule != 0, f->lx_ilp)
                         : select_texplicit(xdt, f->accum, f->K, f->zero_rule != 0, f->lx_ilp, rx.b8 != 0);
    int rc = ensure_lds_attr(d.device, fn);
    if (rc) return rc;
    const int64_t grid = (rows + R - 1) / R;
    if (grid > 0x7fffffff) return fail(TI_ERR_INVALID, "too many rows for one launch");
    const int block = f->tx8 == 3 ? 2 * R : R;   // two lanes a row: 2R threads
    if (block > 512) return fail(TI_ERR_UNSUPPORTED, "two-lane walk needs tiles of <= 256 rows");
    occ_note(fn, block, lds);
  hipLaunchKernelGGL(fn, dim3(static_cast<unsigned>(grid)), dim3(block), lds, stream, a);
    TI_HIP(hipGetLastError());
    return TI_OK;
  } else if (f->layout == 8) {
    const int ii = xdt == TI_F64 ? 1 : 0;
    const ti_forest::RecExplicit& rx = f->rx[ii];
    a.rx_recs = d.rx_recs[ii];
    a.rx_base = d.rx_base;
    a.rx_nint = d.rx_nint;
    a.leaf_base = d.leaf_base;
    a.rx_slots = static_cast<uint32_t>(f->rx_slots);
    a.leaves = d.leaves;
    a.exp_leaf_ids = d.exp_leaf_ids;
    a.bin_tbl = d.bx_tbl[ii];
    a.bin_L = rx.L;
    a.bin_kary = rx.kary;
    a.bin_words = rx.words;
    a.trees = reinterpret_cast<const unsigned char*>(d.hx_top[ii]);
    a.depth = f->hx_top;
    a.tree_stride = static_cast<int64_t>(8) << f->hx_top;   // 2^(D0+1) u32
    a.stage_trees = f->hx_stage;
    a.stage_off = static_cast<int32_t>(align16(feat_bytes + 4));
    lds = static_cast<size_t>(a.stage_off) + static_cast<size_t>(f->hx_stage) * a.tree_stride;
    if (lds > kLdsPerCu || static_cast<int64_t>(kHxPf) * 16 * R < f->hx_stage * a.tree_stride)
      return fail(TI_ERR_UNSUPPORTED, "heap-top layout exceeds LDS");
    a.bin_chunk = bin_chunk_for(static_cast<size_t>(f->hx_stage) * a.tree_stride, R, xdt, f->F);
    KernelFn fn = select_hexplicit(xdt, f->accum, f->K, f->zero_rule != 0, f->hx_ilp);
    int rc = ensure_lds_attr(d.device, fn);
    if (rc) return rc;
    const int64_t grid = (rows + R - 1) / R;
    if (grid > 0x7fffffff) return fail(TI_ERR_INVALID, "too many rows for one launch");
    occ_note(fn, R, lds);
  hipLaunchKernelGGL(fn, dim3(static_cast<unsigned>(grid)), dim3(R), lds, stream, a);
    TI_HIP(hipGetLastError());
    return TI_OK;
  } else {
    a.nodes = d.nodes;
    a.thr64 = d.thr64;
    a.node_base = d.node_base;
    a.root = d.root;
    a.leaf_base = d.leaf_base;
    a.leaves = d.leaves;
    a.exp_leaf_ids = d.exp_leaf_ids;
    a.cat_words = d.cat_words;
  }
  KernelFn fn = select_kernel(f->layout, xdt, f->accum, f->K, feat_lds, f->zero_rule != 0);
  int rc = ensure_lds_attr(d.device, fn);
  if (rc) return rc;
  const int64_t grid = (rows + R - 1) / R;
  if (grid > 0x7fffffff) return fail(TI_ERR_INVALID, "too many rows for one launch");
  occ_note(fn, R, lds);
  hipLaunchKernelGGL(fn, dim3(static_cast<unsigned>(grid)), dim3(R), lds, stream, a);
  TI_HIP(hipGetLastError());
  return TI_OK;
}

// Scratch buffers grow geometrically (x2, >= 4 MiB) so a serving process
// stops reallocating after its first few batch sizes.
int grow(void** buf, size_t* cap, size_t need, bool pinned = false) {
  if (need <= *cap) return TI_OK;
  const size_t n = std::max({need, static_cast<size_t>(4) << 20, 2 * *cap});
  if (*buf) (void)(pinned ? hipHostFree(*buf) : hipFree(*buf));
  *buf = nullptr;
  *cap = 0;
  if (pinned) {
    TI_HIP(hipHostMalloc(buf, n, hipHostMallocDefault));
  } else {
    TI_HIP(hipMalloc(buf, n));
  }
  *cap = n;
  return TI_OK;
}

int launch_any(ti_forest* f, int slot, const void* X, int xdt, int64_t rows, int32_t cols,
               int64_t stride, int kind, void* out, hipStream_t stream);

// Host copies into / out of pinned staging: large copies split over threads
// (one thread moves ~10 GB/s from pageable memory; PCIe Gen5 x16 takes ~55).
void copy_parallel(void* dst, const void* src, size_t n) {
  constexpr size_t kPerThread = 8u << 20;
  const size_t want = std::min<size_t>(8, n / kPerThread);
  if (want < 2) {
    std::memcpy(dst, src, n);
    return;
  }
  std::vector<std::thread> th;
  const size_t part = (n / want + 63) & ~size_t(63);
  for (size_t i = 0; i < want; ++i) {
    const size_t lo = i * part;
    if (lo >= n) break;
    const size_t len = std::min(part, n - lo);
    th.emplace_back([=]() {
      std::memcpy(static_cast<unsigned char*>(dst) + lo, static_cast<const unsigned char*>(src) + lo, len);
    });
  }
  for (auto& t : th) t.join();
}

// Rows per chunk of the host pipeline: TI_CHUNK_MB (default 64) of input,
// a multiple of 512 rows (whole tiles).
int64_t chunk_rows(size_t row_bytes) {
  const int mb = env_int("TI_CHUNK_MB", 64);
  int64_t r = static_cast<int64_t>((static_cast<size_t>(std::max(mb, 1)) << 20) / std::max<size_t>(row_bytes, 1));
  r = std::max<int64_t>(512, r & ~int64_t(511));
  return r;
}

// Batches larger than one chunk: chunks alternate between two lanes (streams
// with their own pinned and device buffers).  While lane A runs chunk c
// (H2D -> kernel -> D2H), the host copies chunk c+1 into lane B's pinned
// buffer and enqueues it, so B's H2D overlaps A's kernel; before lane A takes
// chunk c+2 the host waits for chunk c and copies its result out.  Pinned
// memory is 2 x (chunk in + chunk out) whatever the batch size.
int predict_pipelined(ti_forest* f, int slot, DeviceForest& d, const unsigned char* X, int xdt,
                      int64_t rows, int32_t cols, int64_t stride, int kind, unsigned char* out,
                      int64_t ch) {
  const size_t xs = dtype_size(xdt);
  const size_t os = dtype_size(output_dtype(f, kind)) * output_width(f, kind);
  const size_t x_row = static_cast<size_t>(stride) * xs;
  const size_t x_cap = static_cast<size_t>(ch) * x_row;
  const size_t o_cap = static_cast<size_t>(ch) * os;
  // Whatever path leaves this function (an early TI_HIP return or a failed
  // launch included), no copy or kernel queued on a lane outlives it: the
  // next call reuses -- or frees -- the lane buffers that work reads and writes.
  struct LaneSync {
    DeviceForest& d;
    ~LaneSync() {
      for (int l = 0; l < 2; ++l)
        if (d.lane_stream[l]) (void)hipStreamSynchronize(d.lane_stream[l]);
    }
  } lane_sync{d};
  if (d.lane_x_cap < x_cap || d.lane_o_cap < o_cap) {
    for (int l = 0; l < 2; ++l) {
      if (d.lane_hx[l]) (void)hipHostFree(d.lane_hx[l]);
      if (d.lane_ho[l]) (void)hipHostFree(d.lane_ho[l]);
      if (d.lane_dx[l]) (void)hipFree(d.lane_dx[l]);
      if (d.lane_do[l]) (void)hipFree(d.lane_do[l]);
      d.lane_hx[l] = d.lane_ho[l] = d.lane_dx[l] = d.lane_do[l] = nullptr;
    }
    d.lane_x_cap = d.lane_o_cap = 0;
    for (int l = 0; l < 2; ++l) {
      TI_HIP(hipHostMalloc(&d.lane_hx[l], x_cap, hipHostMallocDefault));
      TI_HIP(hipHostMalloc(&d.lane_ho[l], o_cap, hipHostMallocDefault));
      TI_HIP(hipMalloc(&d.lane_dx[l], x_cap));
      TI_HIP(hipMalloc(&d.lane_do[l], o_cap));
    }
    d.lane_x_cap = x_cap;
    d.lane_o_cap = o_cap;
  }
  for (int l = 0; l < 2; ++l)
    if (!d.lane_stream[l]) TI_HIP(hipStreamCreateWithFlags(&d.lane_stream[l], hipStreamNonBlocking));
  const int64_t n_chunks = (rows + ch - 1) / ch;
  int64_t pending[2] = {-1, -1};   // chunk whose result lane l still holds
  auto drain = [&](int l) -> int {
    if (pending[l] < 0) return TI_OK;
    TI_HIP(hipStreamSynchronize(d.lane_stream[l]));
    const int64_t c = pending[l];
    const int64_t n = std::min(ch, rows - c * ch);
    copy_parallel(out + static_cast<size_t>(c * ch) * os, d.lane_ho[l], static_cast<size_t>(n) * os);
    pending[l] = -1;
    return TI_OK;
  };
  int rc = TI_OK;
  for (int64_t c = 0; c < n_chunks && rc == TI_OK; ++c) {
    const int l = static_cast<int>(c & 1);
    if ((rc = drain(l))) break;
    const int64_t r0 = c * ch;
    const int64_t n = std::min(ch, rows - r0);
    const size_t xb = static_cast<size_t>((n - 1) * stride + cols) * xs;
    copy_parallel(d.lane_hx[l], X + static_cast<size_t>(r0) * x_row, xb);
    hipStream_t st = d.lane_stream[l];
    TI_HIP(hipMemcpyAsync(d.lane_dx[l], d.lane_hx[l], xb, hipMemcpyHostToDevice, st));
    if ((rc = launch_any(f, slot, d.lane_dx[l], xdt, n, cols, stride, kind, d.lane_do[l], st)))
      break;
    TI_HIP(hipMemcpyAsync(d.lane_ho[l], d.lane_do[l], static_cast<size_t>(n) * os,
                          hipMemcpyDeviceToHost, st));
    pending[l] = c;
  }
  // the other lane first: it holds the older chunk
  const int last = static_cast<int>((n_chunks - 1) & 1);
  const int r1 = drain(last ^ 1);
  const int r2 = drain(last);
  return rc ? rc : (r1 ? r1 : r2);
}

// A caller's host span page-locked for one call (hipHostRegister over its
// page-rounded range) and unlocked when this goes out of scope.  Only a
// registration this call made counts: pages that another registration already
// holds (hipErrorHostMemoryAlreadyRegistered) may be unlocked by their owner
// mid-DMA, so reg() reports failure and the caller takes the staging chunks.
struct HostSpan {
  void* p = nullptr;
  bool mine = false;
  bool reg(const void* base, size_t n, bool portable = false) {
    const uintptr_t pg = 4096;
    const uintptr_t lo = reinterpret_cast<uintptr_t>(base) & ~(pg - 1);
    const uintptr_t hi = (reinterpret_cast<uintptr_t>(base) + n + pg - 1) & ~(pg - 1);
    p = reinterpret_cast<void*>(lo);
    const hipError_t e = hipHostRegister(p, hi - lo, portable ? hipHostRegisterPortable
                                                                : hipHostRegisterDefault);
    if (e == hipSuccess) {
      mine = true;
      return true;
    }
    (void)hipGetLastError();
    return false;
  }
  ~HostSpan() {
    if (mine) (void)hipHostUnregister(p);
  }
};

// The caller's own buffers page-locked for the call (hipHostRegister), so
// chunks go H2D straight from X and D2H straight into out, alternating two
// lanes with no host copy and no host wait until the end (TI_OPT_HOST_REGISTER;
// A/B against the pinned-chunk pipeline, which copies every byte once on the
// host).  Returns TI_ERR_UNSUPPORTED, having done nothing, when a buffer
// cannot be registered; the caller then takes the pinned-chunk pipeline.
// `pre`: the caller registered X and out already (the multi-device ti_predict
// registers the whole batch once, before its shard threads start).
int predict_registered(ti_forest* f, int slot, DeviceForest& d, const unsigned char* X, int xdt,
                       int64_t rows, int32_t cols, int64_t stride, int kind, unsigned char* out,
                       int64_t ch, bool pre) {
  const size_t xs = dtype_size(xdt);
  const size_t os = dtype_size(output_dtype(f, kind)) * output_width(f, kind);
  const size_t x_row = static_cast<size_t>(stride) * xs;
  const size_t x_bytes = static_cast<size_t>((rows - 1) * stride + cols) * xs;
  const size_t o_bytes = static_cast<size_t>(rows) * os;
  HostSpan rx, ro;
  if (!pre && (!rx.reg(X, x_bytes) || !ro.reg(out, o_bytes))) return TI_ERR_UNSUPPORTED;
  struct LaneSync {
    DeviceForest& d;
    ~LaneSync() {
      for (int l = 0; l < 2; ++l)
        if (d.lane_stream[l]) (void)hipStreamSynchronize(d.lane_stream[l]);
    }
  } lane_sync{d};
  const size_t x_cap = static_cast<size_t>(ch) * x_row;
  const size_t o_cap = static_cast<size_t>(ch) * os;
  if (d.lane_x_cap < x_cap || d.lane_o_cap < o_cap) {
    for (int l = 0; l < 2; ++l) {
      if (d.lane_hx[l]) (void)hipHostFree(d.lane_hx[l]);
      if (d.lane_ho[l]) (void)hipHostFree(d.lane_ho[l]);
      if (d.lane_dx[l]) (void)hipFree(d.lane_dx[l]);
      if (d.lane_do[l]) (void)hipFree(d.lane_do[l]);
      d.lane_hx[l] = d.lane_ho[l] = d.lane_dx[l] = d.lane_do[l] = nullptr;
    }
    d.lane_x_cap = d.lane_o_cap = 0;
    for (int l = 0; l < 2; ++l) {
      TI_HIP(hipHostMalloc(&d.lane_hx[l], x_cap, hipHostMallocDefault));
      TI_HIP(hipHostMalloc(&d.lane_ho[l], o_cap, hipHostMallocDefault));
      TI_HIP(hipMalloc(&d.lane_dx[l], x_cap));
      TI_HIP(hipMalloc(&d.lane_do[l], o_cap));
    }
    d.lane_x_cap = x_cap;
    d.lane_o_cap = o_cap;
  }
  for (int l = 0; l < 2; ++l)
    if (!d.lane_stream[l]) TI_HIP(hipStreamCreateWithFlags(&d.lane_stream[l], hipStreamNonBlocking));
  const int64_t n_chunks = (rows + ch - 1) / ch;
  for (int64_t c = 0; c < n_chunks; ++c) {
    const int l = static_cast<int>(c & 1);
    const int64_t r0 = c * ch;
    const int64_t n = std::min(ch, rows - r0);
    const size_t xb = static_cast<size_t>((n - 1) * stride + cols) * xs;
    hipStream_t st = d.lane_stream[l];
    TI_HIP(hipMemcpyAsync(d.lane_dx[l], X + static_cast<size_t>(r0) * x_row, xb,
                          hipMemcpyHostToDevice, st));
    int rc = launch_any(f, slot, d.lane_dx[l], xdt, n, cols, stride, kind, d.lane_do[l], st);
    if (rc) return rc;
    TI_HIP(hipMemcpyAsync(out + static_cast<size_t>(r0) * os, d.lane_do[l], static_cast<size_t>(n) * os,
                          hipMemcpyDeviceToHost, st));
  }
  for (int l = 0; l < 2; ++l) TI_HIP(hipStreamSynchronize(d.lane_stream[l]));
  return TI_OK;
}

// reg: 0 pinned staging chunks; 1 page-lock this shard's X and out for the
// call (one device); 2 the caller page-locked the whole batch (multi-device)
int predict_shard(ti_forest* f, int slot, DeviceForest& d, const unsigned char* X, int xdt,
                  int64_t rows, int32_t cols, int64_t stride, int kind, unsigned char* out,
                  int reg) {
  std::lock_guard<std::mutex> lk(d.mu);
  TI_HIP(hipSetDevice(d.device));
  {
    const int64_t ch = chunk_rows(static_cast<size_t>(stride) * dtype_size(xdt));
    if (rows > ch) {
      if (reg) {
        const int rc = predict_registered(f, slot, d, X, xdt, rows, cols, stride, kind, out, ch,
                                          reg == 2);
        if (rc != TI_ERR_UNSUPPORTED) return rc;
      }
      return predict_pipelined(f, slot, d, X, xdt, rows, cols, stride, kind, out, ch);
    }
  }
  const size_t xs = dtype_size(xdt);
  const size_t x_elems = static_cast<size_t>((rows - 1) * stride + cols);
  const size_t out_bytes = static_cast<size_t>(rows * output_width(f, kind)) *
                           dtype_size(output_dtype(f, kind));
  int rc;
  const size_t x_bytes = x_elems * xs;
  if ((rc = grow(&d.x_buf, &d.x_cap, x_bytes))) return rc;
  if ((rc = grow(&d.out_buf, &d.out_cap, out_bytes))) return rc;
  if ((rc = grow(&d.hx_pin, &d.hx_cap, x_bytes, true))) return rc;
  if ((rc = grow(&d.ho_pin, &d.ho_cap, out_bytes, true))) return rc;
  // caller memory -> pinned staging -> DMA; keeps H2D/D2H asynchronous and at
  // PCIe rate whatever kind of host memory the caller holds
  copy_parallel(d.hx_pin, X, x_bytes);
  TI_HIP(hipMemcpyAsync(d.x_buf, d.hx_pin, x_bytes, hipMemcpyHostToDevice, d.stream));
  if ((rc = launch_any(f, slot, d.x_buf, xdt, rows, cols, stride, kind, d.out_buf, d.stream)))
    return rc;
  TI_HIP(hipMemcpyAsync(d.ho_pin, d.out_buf, out_bytes, hipMemcpyDeviceToHost, d.stream));
  TI_HIP(hipStreamSynchronize(d.stream));
  copy_parallel(out, d.ho_pin, out_bytes);
  return TI_OK;
}

// ------------------------------------------------- more than 16 output groups
// Output transform over [rows, K] margins for forests split into group parts
// (the fused epilogue covers K <= kMaxGroups).  Same arithmetic as
// ti::finish_row: softmax with the maximum in ACC and the sum in double,
// first-maximum argmax.
template <typename ACC>
__global__ void transform_rows_kernel(const ACC* __restrict__ m, int64_t rows, int K, int tr,
                                      double param, ACC* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  const ACC* v = m + r * K;
  if (tr == TI_TRANSFORM_ARGMAX) {
    int best = 0;
    for (int k = 1; k < K; ++k)
      if (v[best] < v[k]) best = k;
    out[r] = (ACC)best;
    return;
  }
  ACC* o = out + r * K;
  if (tr == TI_TRANSFORM_SOFTMAX) {
    ACC wmax = v[0];
    for (int k = 1; k < K; ++k) wmax = (v[k] < wmax) ? wmax : v[k];
    double wsum = 0.0;
    for (int k = 0; k < K; ++k) wsum += ti::t_exp(v[k] - wmax);
    for (int k = 0; k < K; ++k) o[k] = ti::t_exp(v[k] - wmax) / (ACC)wsum;
    return;
  }
  for (int k = 0; k < K; ++k) {
    ACC x = v[k];
    switch (tr) {
      case TI_TRANSFORM_SIGMOID: x = ACC(1) / (ACC(1) + ti::t_exp(-((ACC)param * x))); break;
      case TI_TRANSFORM_HINGE: x = x > ACC(0) ? ACC(1) : ACC(0); break;
      case TI_TRANSFORM_EXP: x = ti::t_exp(x); break;
      case TI_TRANSFORM_SIGNSQUARE: x = (ACC)((x > ACC(0)) - (x < ACC(0))) * x * x; break;
      case TI_TRANSFORM_LOG1PEXP: x = ti::t_log1p(ti::t_exp(x)); break;
      case TI_TRANSFORM_STEP: x = x >= ACC(0) ? ACC(1) : ACC(0); break;
      default: break;
    }
    o[k] = x;
  }
}

// dst[r, map[j]] = src[r, j] for the leaf-id columns of one part.
__global__ void scatter_cols_kernel(const int32_t* __restrict__ src, int64_t rows, int tc,
                                    const int32_t* __restrict__ map, int T,
                                    int32_t* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * tc) return;
  const int64_t r = i / tc;
  const int j = (int)(i - r * tc);
  dst[r * T + map[j]] = src[i];
}

int launch_any(ti_forest* f, int slot, const void* X, int xdt, int64_t rows, int32_t cols,
               int64_t stride, int kind, void* out, hipStream_t stream);

// Device path of a chunked forest: each part writes its margin columns (or
// leaf-id columns) through a stream-ordered scratch buffer, then the output
// transform runs over the assembled [rows, K] margins.
int launch_chunked(ti_forest* f, int slot, const void* X, int xdt, int64_t rows, int32_t cols,
                   int64_t stride, int kind, void* out, hipStream_t stream) {
  const size_t as = f->accum == TI_F64 ? 8 : 4;
  const int threads = 256;
  if (kind == TI_OUTPUT_LEAF && f->LW != 1)   // vector leaves: every part holds every tree
    return launch_any(f->parts[0].get(), slot, X, xdt, rows, cols, stride, kind, out, stream);
  void* tmp = nullptr;
  void* marg = nullptr;
  int32_t* dmap = nullptr;
  int rc = TI_OK;
  size_t tmp_bytes = 0;
  const int64_t cw = kind == TI_OUTPUT_CONTRIB ? f->F + 1 : 1;   // columns per group
  for (auto& p : f->parts)
    tmp_bytes = std::max(tmp_bytes, static_cast<size_t>(rows) *
                                        (kind == TI_OUTPUT_LEAF ? 4 * p->T : as * p->K * cw));
  TI_HIP(hipMallocAsync(&tmp, tmp_bytes, stream));
  const bool transform = kind == TI_OUTPUT_PREDICT && f->transform != TI_TRANSFORM_IDENTITY;
  if (transform) {
    if (hipMallocAsync(&marg, static_cast<size_t>(rows) * f->K * as, stream) != hipSuccess) {
      (void)hipFreeAsync(tmp, stream);
      return fail(TI_ERR_NOMEM, "margin scratch allocation failed");
    }
  }
  void* mdst = transform ? marg : out;
  for (size_t c = 0; c < f->parts.size() && rc == TI_OK; ++c) {
    ti_forest* p = f->parts[c].get();
    if (kind == TI_OUTPUT_LEAF) {
      rc = launch_any(p, slot, X, xdt, rows, cols, stride, kind, tmp, stream);
      if (rc) break;
      const std::vector<int32_t>& map = f->part_trees[c];
      if (hipMallocAsync(reinterpret_cast<void**>(&dmap), map.size() * 4, stream) != hipSuccess ||
          hipMemcpyAsync(dmap, map.data(), map.size() * 4, hipMemcpyHostToDevice, stream) !=
              hipSuccess) {
        rc = fail(TI_ERR_DEVICE, "leaf map upload failed");
        break;
      }
      const int64_t n = rows * p->T;
      hipLaunchKernelGGL(scatter_cols_kernel, dim3(static_cast<unsigned>((n + threads - 1) / threads)),
                         dim3(threads), 0, stream, static_cast<const int32_t*>(tmp), rows, p->T,
                         dmap, f->T, static_cast<int32_t*>(out));
      (void)hipFreeAsync(dmap, stream);
      dmap = nullptr;
    } else {
      const int pk = kind == TI_OUTPUT_CONTRIB ? TI_OUTPUT_CONTRIB : TI_OUTPUT_MARGIN;
      rc = launch_any(p, slot, X, xdt, rows, cols, stride, pk, tmp, stream);
      if (rc) break;
      if (hipMemcpy2DAsync(static_cast<unsigned char*>(mdst) + f->part_k0[c] * cw * as,
                           f->K * cw * as, tmp, p->K * cw * as, p->K * cw * as, rows,
                           hipMemcpyDeviceToDevice, stream) != hipSuccess)
        rc = fail(TI_ERR_DEVICE, "margin column copy failed");
    }
  }
  if (rc == TI_OK && transform) {
    const unsigned grid = static_cast<unsigned>((rows + threads - 1) / threads);
    if (f->accum == TI_F64)
      hipLaunchKernelGGL(transform_rows_kernel<double>, dim3(grid), dim3(threads), 0, stream,
                         static_cast<const double*>(marg), rows, f->K, f->transform, f->tparam,
                         static_cast<double*>(out));
    else
      hipLaunchKernelGGL(transform_rows_kernel<float>, dim3(grid), dim3(threads), 0, stream,
                         static_cast<const float*>(marg), rows, f->K, f->transform, f->tparam,
                         static_cast<float*>(out));
    if (hipGetLastError() != hipSuccess) rc = fail(TI_ERR_DEVICE, "transform launch failed");
  }
  (void)hipFreeAsync(tmp, stream);
  if (marg) (void)hipFreeAsync(marg, stream);
  return rc;
}

// TI_OUTPUT_CONTRIB on one (unchunked) forest.  contrib_reg_kernel when the
// row's accumulators fit LDS (K * (F + 1) <= kShapLdsW) and paths have <= 32
// unique features: path slices over blockIdx.y, partials summed in slice
// order by contrib_slices_kernel.  Otherwise contrib_kernel, whose float32
// forests accumulate in a float64 scratch.
// First contributions call: build the path tables on the host and upload them
// to every device replica (under the forest's lock; later calls see
// shap_ready and skip it).
int ensure_shap(ti_forest* f) {
  if (f->shap_ready.load(std::memory_order_acquire)) return TI_OK;
  std::lock_guard<std::mutex> lk(f->shap_mu);
  if (f->shap_ready.load(std::memory_order_relaxed)) return TI_OK;
  if (f->h_paths.empty()) build_shap(&f->shap_src->desc, f);
  // the coefficient table's shape (contrib_reg_kernel TAB): paths of <= 8
  // unique features, 2^n x 8 coefficients each (padded), in the path
  // arithmetic's type.  The table itself is built per replica, later, by
  // ensure_shap_table.
  {
    const int mt = (f->accum != TI_F64 && !env_int("TI_SHAP_F64", 0)) ? 4 : 8;
    const int64_t W = static_cast<int64_t>(f->K) * (f->F + 1);
    f->h_tab_off.assign(f->h_paths.size(), 0);
    int64_t len = 0;
    bool ok = W <= kShapLdsW && f->shap_maxl <= kShapTabStride && !f->h_paths.empty();
    for (size_t i = 0; ok && i < f->h_paths.size(); ++i) {
      f->h_tab_off[i] = len;
      len += (int64_t(1) << f->h_paths[i].n) * kShapTabStride;
    }
    f->shap_tab_mt = ok ? mt : 0;
    f->shap_tab_len = ok ? len : 0;
    if (!ok) f->h_tab_off.clear();
  }
  int dev0 = 0;
  TI_HIP(hipGetDevice(&dev0));
  int rc = TI_OK;
  // each replica's byte count before the uploads: a failure restores it, so
  // ti_forest_info's device_bytes does not keep the freed tables
  std::vector<int64_t> bytes0;
  for (auto& dp : f->devs) bytes0.push_back(dp->bytes);
  for (auto& dp : f->devs) {
    DeviceForest& d = *dp;
    if ((rc = fail_hip(hipSetDevice(d.device), "hipSetDevice"))) break;
    if ((rc = upload(&d.shap_paths, f->h_paths, &d.bytes)) ||
        (rc = upload(&d.shap_elems, f->h_elems, &d.bytes)) ||
        (rc = upload(&d.shap_leaf, f->h_path_leaf, &d.bytes)) ||
        (rc = upload(&d.shap_bias, f->h_shap_bias, &d.bytes)))
      break;
  }
  if (rc) {
    // nothing half-built survives: every replica's path tables are freed (the
    // host tables stay, so the next call retries from them)
    const std::string err = g_last_error;
    for (size_t i = 0; i < f->devs.size(); ++i) {
      (void)hipSetDevice(f->devs[i]->device);
      free_shap(*f->devs[i]);
      f->devs[i]->bytes = bytes0[i];
    }
    (void)hipGetLastError();
    (void)hipSetDevice(dev0);
    return fail(rc, err);
  }
  TI_HIP(hipSetDevice(dev0));
  f->h_paths.clear(); f->h_paths.shrink_to_fit();
  f->h_elems.clear(); f->h_elems.shrink_to_fit();
  f->h_path_leaf.clear(); f->h_path_leaf.shrink_to_fit();
  f->shap_src.reset();
  f->shap_ready.store(true, std::memory_order_release);
  return TI_OK;
}

// The coefficient table of one replica (device d.device current), built on
// the first contributions batch that would use it.  It is an optimisation
// only: any failure (over the size cap, allocation, launch) frees what was
// allocated, clears the HIP error and marks the replica, whose contributions
// then take the extend / unwind kernel -- never an error for the caller.  The
// build runs on a private stream and waits for that stream alone.
void ensure_shap_table(ti_forest* f, DeviceForest& d) {
  std::lock_guard<std::mutex> lk(f->shap_mu);
  if (d.shap_tab_state != 0) return;
  d.shap_tab_state = -1;
  const size_t bytes = static_cast<size_t>(f->shap_tab_len) * f->shap_tab_mt;
  if (!f->shap_tab_mt || f->shap_tab_mb <= 0 ||
      bytes > (static_cast<size_t>(f->shap_tab_mb) << 20))
    return;
  const auto t0 = std::chrono::steady_clock::now();
  hipStream_t s = nullptr;
  bool ok = hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess;
  int64_t up = 0;
  ok = ok && !env_int("TI_SHAP_TABLE_FAULT", 0) &&   // fault injection (tests)
       upload(&d.shap_tab_off, f->h_tab_off, &up) == TI_OK &&
       hipMalloc(&d.shap_tab, std::max<size_t>(bytes, 16)) == hipSuccess;
  if (ok) {
    const unsigned np = static_cast<unsigned>(f->h_tab_off.size());
    if (f->shap_tab_mt == 4)
      hipLaunchKernelGGL((shap_table_kernel<float, 16>), dim3(np), dim3(256), 0, s,
                         d.shap_paths, d.shap_elems, d.shap_tab_off, static_cast<float*>(d.shap_tab));
    else
      hipLaunchKernelGGL((shap_table_kernel<double, 16>), dim3(np), dim3(256), 0, s,
                         d.shap_paths, d.shap_elems, d.shap_tab_off, static_cast<double*>(d.shap_tab));
    ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(s) == hipSuccess;
  }
  if (s) (void)hipStreamDestroy(s);
  if (!ok) {
    if (d.shap_tab) (void)hipFree(d.shap_tab);
    if (d.shap_tab_off) (void)hipFree(d.shap_tab_off);
    d.shap_tab = nullptr;
    d.shap_tab_off = nullptr;
    (void)hipGetLastError();
    return;
  }
  d.bytes += up + static_cast<int64_t>(bytes);
  d.shap_tab_state = 1;
  f->shap_tab_build_ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int launch_contrib(ti_forest* f, DeviceForest& d, const void* X, int xdt, int64_t rows,
                   int32_t cols, int64_t stride, void* out, hipStream_t stream) {
  if (!f->has_shap)
    return fail(TI_ERR_UNSUPPORTED,
                "contributions need node covers (ti_forest_desc.cover) and no categorical splits");
  {
    const int rc = ensure_shap(f);
    if (rc) return rc;
  }
  const int64_t W = static_cast<int64_t>(f->K) * (f->F + 1);
  const int64_t n_paths = static_cast<int64_t>(d.shap_paths ? 1 : 0) * f->shap_npaths;
  const int force_generic = env_int("TI_SHAP_GENERIC", 0);
  if (W <= kShapLdsW && f->shap_maxl <= 32 && !force_generic) {
    // registers + LDS accumulators: no scratch accumulator, no memset
    const int maxn = f->shap_maxl <= 8 ? 8 : f->shap_maxl <= 16 ? 16 : 32;
    const int force_f64 = env_int("TI_SHAP_F64", 0);
    const bool f32_math = f->accum != TI_F64 && !force_f64;
    const size_t lds_w = static_cast<size_t>(W) * 64 * (f32_math ? 4 : 8);
    const unsigned grid_r = static_cast<unsigned>((rows + 63) / 64);
    if (rows == 0) return TI_OK;
    // Path slices: one 64-row wave walks n_paths / slices paths, so a small
    // batch still fills the 256 CUs (>= kShapWaveTarget waves); partials
    // [slices][W][rows] are summed in slice order by contrib_slices_kernel.
    const int force_slices = env_int("TI_SHAP_SLICES", 0);
    int64_t slices = force_slices > 0 ? force_slices
                                      : (kShapWaveTarget + grid_r - 1) / static_cast<int64_t>(grid_r);
    slices = std::min<int64_t>(slices, std::max<int64_t>(1, n_paths / kShapMinPathsPerSlice));
    slices = std::min<int64_t>(slices, kShapMaxSlices);
    while (slices > 1 && static_cast<uint64_t>(slices) * W * rows * 8 > kShapPartBytesMax) --slices;
    slices = std::max<int64_t>(slices, 1);
    const int64_t pps = (n_paths + slices - 1) / slices;
    // the coefficient table pays off for small batches (C2 model: 4,096 rows
    // 4.1e5 vs 2.7e5 rows/s); at 100k rows its gathers (a 64-row wave reads
    // most of each path's 2^n x 32 B block) make it slower than the extend /
    // unwind arithmetic (2.2e5 vs 2.9e5): profiles/r3_shap_table.jsonl
    const bool want_tab = f->shap_tab_mt != 0 && rows <= f->shap_tab_rows;
    if (want_tab && d.shap_tab_state == 0) ensure_shap_table(f, d);
    double* part = nullptr;
    if (slices > 1)
      TI_HIP(hipMallocAsync(reinterpret_cast<void**>(&part),
                            static_cast<size_t>(slices * W * rows) * 8, stream));
#define TI_CONTRIB_REG(XT_, ACC_, MT_, N_)                                                          \
  do {                                                                                         \
    const bool tab_ = want_tab && d.shap_tab_state == 1 &&                                     \
                      f->shap_tab_mt == (int)sizeof(MT_);                                      \
    KernelFn fn_ = tab_ ? reinterpret_cast<KernelFn>(contrib_reg_kernel<XT_, ACC_, MT_, 8, true>) \
                        : reinterpret_cast<KernelFn>(contrib_reg_kernel<XT_, ACC_, MT_, N_>);  \
    int rc_ = ensure_lds_attr(d.device, fn_);                                                  \
    if (rc_) return rc_;                                                                       \
    if (tab_)                                                                                  \
      hipLaunchKernelGGL((contrib_reg_kernel<XT_, ACC_, MT_, 8, true>), dim3(grid_r, (unsigned)slices), \
                         dim3(64), lds_w, stream,                                              \
                         static_cast<const XT_*>(X), rows, stride, cols, f->lgb_zero_map,      \
                         d.shap_paths, n_paths, d.shap_elems, d.shap_leaf, f->LW, f->K, f->F,  \
                         f->shap_maxl, d.shap_bias, f->divisor, part, pps, static_cast<ACC_*>(out), \
                         static_cast<const MT_*>(d.shap_tab), d.shap_tab_off);                 \
    else                                                                                       \
      hipLaunchKernelGGL((contrib_reg_kernel<XT_, ACC_, MT_, N_>), dim3(grid_r, (unsigned)slices), dim3(64), \
                         lds_w, stream,                                                        \
                         static_cast<const XT_*>(X), rows, stride, cols, f->lgb_zero_map,      \
                         d.shap_paths, n_paths, d.shap_elems, d.shap_leaf, f->LW, f->K, f->F,  \
                         f->shap_maxl, d.shap_bias, f->divisor, part, pps, static_cast<ACC_*>(out), \
                         static_cast<const MT_*>(nullptr), static_cast<const int64_t*>(nullptr)); \
    if (part) {                                                                                \
      const unsigned g2 = static_cast<unsigned>((rows + 255) / 256);                           \
      hipLaunchKernelGGL((contrib_slices_kernel<ACC_>), dim3(g2), dim3(256), 0, stream, part,  \
                         (int32_t)slices, rows, f->K, f->F, d.shap_bias, f->divisor,           \
                         static_cast<ACC_*>(out));                                             \
    }                                                                                          \
  } while (0)
#define TI_CONTRIB_REG_N(XT_, ACC_, MT_)                     \
  do {                                                       \
    if (maxn == 8) TI_CONTRIB_REG(XT_, ACC_, MT_, 8);        \
    else if (maxn == 16) TI_CONTRIB_REG(XT_, ACC_, MT_, 16); \
    else TI_CONTRIB_REG(XT_, ACC_, MT_, 32);                 \
  } while (0)
    // Path arithmetic in the forest's accumulator type: float64 for LightGBM
    // and sklearn; float32 for XGBoost, whose TreeShap keeps its path
    // elements and contributions in bst_float (TI_SHAP_F64=1 forces
    // float64).  Each slice accumulates in that type in LDS (float32 halves
    // the LDS per workgroup: 2x workgroups per CU); slices sum in float64.
    if (xdt == TI_F32) {
      if (f->accum == TI_F64) TI_CONTRIB_REG_N(float, double, double);
      else if (f32_math) TI_CONTRIB_REG_N(float, float, float);
      else TI_CONTRIB_REG_N(float, float, double);
    } else {
      if (f->accum == TI_F64) TI_CONTRIB_REG_N(double, double, double);
      else if (f32_math) TI_CONTRIB_REG_N(double, float, float);
      else TI_CONTRIB_REG_N(double, float, double);
    }
#undef TI_CONTRIB_REG_N
#undef TI_CONTRIB_REG
    TI_HIP(hipGetLastError());
    if (part) TI_HIP(hipFreeAsync(part, stream));
    return TI_OK;
  }
  double* acc = nullptr;
  if (f->accum == TI_F64) {
    acc = static_cast<double*>(out);
  } else {
    TI_HIP(hipMallocAsync(reinterpret_cast<void**>(&acc), static_cast<size_t>(rows * W) * 8, stream));
  }
  TI_HIP(hipMemsetAsync(acc, 0, static_cast<size_t>(rows * W) * 8, stream));
  const size_t lds = static_cast<size_t>(2 * f->shap_maxl + 1) * 64 * 8;
  KernelFn fn;
  if (xdt == TI_F32)
    fn = f->accum == TI_F64 ? reinterpret_cast<KernelFn>(contrib_kernel<float, double>)
                            : reinterpret_cast<KernelFn>(contrib_kernel<float, float>);
  else
    fn = f->accum == TI_F64 ? reinterpret_cast<KernelFn>(contrib_kernel<double, double>)
                            : reinterpret_cast<KernelFn>(contrib_kernel<double, float>);
  int rc = ensure_lds_attr(d.device, fn);
  if (rc) return rc;
  const unsigned grid = static_cast<unsigned>((rows + 63) / 64);
  if (xdt == TI_F32) {
    if (f->accum == TI_F64)
      hipLaunchKernelGGL((contrib_kernel<float, double>), dim3(grid), dim3(64), lds, stream,
                         static_cast<const float*>(X), rows, stride, cols, f->lgb_zero_map,
                         d.shap_paths, n_paths, d.shap_elems, d.shap_leaf, f->LW, f->K, f->F,
                         f->shap_maxl, d.shap_bias, f->divisor, acc, static_cast<double*>(out));
    else
      hipLaunchKernelGGL((contrib_kernel<float, float>), dim3(grid), dim3(64), lds, stream,
                         static_cast<const float*>(X), rows, stride, cols, f->lgb_zero_map,
                         d.shap_paths, n_paths, d.shap_elems, d.shap_leaf, f->LW, f->K, f->F,
                         f->shap_maxl, d.shap_bias, f->divisor, acc, static_cast<float*>(out));
  } else {
    if (f->accum == TI_F64)
      hipLaunchKernelGGL((contrib_kernel<double, double>), dim3(grid), dim3(64), lds, stream,
                         static_cast<const double*>(X), rows, stride, cols, f->lgb_zero_map,
                         d.shap_paths, n_paths, d.shap_elems, d.shap_leaf, f->LW, f->K, f->F,
                         f->shap_maxl, d.shap_bias, f->divisor, acc, static_cast<double*>(out));
    else
      hipLaunchKernelGGL((contrib_kernel<double, float>), dim3(grid), dim3(64), lds, stream,
                         static_cast<const double*>(X), rows, stride, cols, f->lgb_zero_map,
                         d.shap_paths, n_paths, d.shap_elems, d.shap_leaf, f->LW, f->K, f->F,
                         f->shap_maxl, d.shap_bias, f->divisor, acc, static_cast<float*>(out));
  }
  TI_HIP(hipGetLastError());
  if (acc != out) TI_HIP(hipFreeAsync(acc, stream));
  return TI_OK;
}

int launch_any(ti_forest* f, int slot, const void* X, int xdt, int64_t rows, int32_t cols,
               int64_t stride, int kind, void* out, hipStream_t stream) {
  if (kind == TI_OUTPUT_CONTRIB && f->parts.empty())
    return launch_contrib(f, *f->devs[slot], X, xdt, rows, cols, stride, out, stream);
  if (!f->parts.empty())
    return launch_chunked(f, slot, X, xdt, rows, cols, stride, kind, out, stream);
  return launch(f, *f->devs[slot], X, xdt, rows, cols, stride, kind, out, stream);
}

// Split a forest of K > kMaxGroups outputs into parts of at most kMaxGroups
// groups.  Scalar leaves (leaf_width 1, XGBoost / LightGBM multiclass): a
// part holds the trees of its groups, in their original order, so each
// group's sum is bit-identical.  Vector leaves (sklearn classifiers): every
// part holds every tree with its slice of the leaf vectors.
int create_chunked(const ti_forest_desc* d, const int32_t* devices, int32_t n_devices,
                   ti_forest** out) {
  std::unique_ptr<ti_forest> f(new ti_forest());
  f->T = d->n_trees;
  f->F = d->n_features;
  f->K = d->n_groups;
  f->LW = d->leaf_width;
  f->accum = d->accum_dtype;
  f->base_first = d->base_first ? 1 : 0;
  f->transform = d->transform;
  f->tparam = d->transform_param;
  f->divisor = d->average_divisor;
  const int K = d->n_groups, LW = d->leaf_width;
  for (int k0 = 0; k0 < K; k0 += ti::kMaxGroups) {
    const int kc = std::min(ti::kMaxGroups, K - k0);
    std::vector<int32_t> trees, tgrp, feat, left, right, leaf_id, cat_nw;
    std::vector<int64_t> toff(1, 0), cat_off;
    std::vector<double> thr, lv, cov, base(d->base_margin + k0, d->base_margin + k0 + kc);
    std::vector<uint8_t> flags;
    for (int t = 0; t < d->n_trees; ++t) {
      if (LW == 1 && (d->tree_group[t] < k0 || d->tree_group[t] >= k0 + kc)) continue;
      trees.push_back(t);
      tgrp.push_back(LW == 1 ? d->tree_group[t] - k0 : 0);
      for (int64_t g = d->tree_offset[t]; g < d->tree_offset[t + 1]; ++g) {
        feat.push_back(d->feature[g]);
        thr.push_back(d->threshold[g]);
        flags.push_back(d->flags[g]);
        left.push_back(d->left[g]);
        right.push_back(d->right[g]);
        leaf_id.push_back(d->leaf_id[g]);
        if (d->cover) cov.push_back(d->cover[g]);
        if (d->cat_offset) {
          cat_off.push_back(d->cat_offset[g]);
          cat_nw.push_back(d->cat_nwords[g]);
        }
        if (LW == 1) {
          lv.push_back(d->leaf_value[g]);
        } else {
          for (int k = 0; k < kc; ++k) lv.push_back(d->leaf_value[g * LW + k0 + k]);
        }
      }
      toff.push_back(static_cast<int64_t>(feat.size()));
    }
    if (trees.empty())
      return fail(TI_ERR_UNSUPPORTED, "output groups " + std::to_string(k0) + ".." +
                                          std::to_string(k0 + kc - 1) + " have no trees");
    ti_forest_desc sd = *d;
    sd.n_trees = static_cast<int32_t>(trees.size());
    sd.n_groups = kc;
    sd.leaf_width = LW == 1 ? 1 : kc;
    sd.n_nodes = static_cast<int64_t>(feat.size());
    sd.tree_offset = toff.data();
    sd.tree_group = tgrp.data();
    sd.feature = feat.data();
    sd.threshold = thr.data();
    sd.flags = flags.data();
    sd.left = left.data();
    sd.right = right.data();
    sd.leaf_id = leaf_id.data();
    sd.leaf_value = lv.data();
    sd.base_margin = base.data();
    sd.transform = TI_TRANSFORM_IDENTITY;
    sd.transform_param = 1.0;
    sd.cat_offset = d->cat_offset ? cat_off.data() : nullptr;
    sd.cat_nwords = d->cat_offset ? cat_nw.data() : nullptr;
    sd.cover = d->cover ? cov.data() : nullptr;
    ti_forest* part = nullptr;
    const int rc = ti_forest_create(&sd, devices, n_devices, &part);
    if (rc) {
      for (auto& q : f->parts) ti_forest_destroy(q.release());
      return rc;
    }
    f->parts.emplace_back(part);
    f->part_k0.push_back(k0);
    f->part_trees.push_back(std::move(trees));
    f->depth = std::max(f->depth, part->depth);
  }
  f->layout = f->parts[0]->layout;
  *out = f.release();
  return TI_OK;
}

// The forest whose DeviceForest (stream, staging buffers, lock) serves a slot.
ti_forest* base_forest(ti_forest* f) {
  while (!f->parts.empty()) f = f->parts[0].get();
  return f;
}

}  // namespace

extern "C" {

int32_t ti_abi_version(void) { return TI_ABI_VERSION; }

const char* ti_last_error(void) { return g_last_error.c_str(); }

int ti_device_count(int32_t* count) {
  if (!count) return fail(TI_ERR_INVALID, "null count");
  int n = 0;
  TI_HIP(hipGetDeviceCount(&n));
  *count = n;
  return TI_OK;
}

int ti_forest_create(const ti_forest_desc* desc, const int32_t* devices, int32_t n_devices,
                     ti_forest** out) {
  if (!out) return fail(TI_ERR_INVALID, "null output handle");
  *out = nullptr;
  if (!devices || n_devices <= 0) return fail(TI_ERR_INVALID, "need at least one device");
  std::vector<int> depth;
  int rc = validate(desc, &depth);
  if (rc) return rc;
  int n_visible = 0;
  TI_HIP(hipGetDeviceCount(&n_visible));
  for (int i = 0; i < n_devices; ++i)
    if (devices[i] < 0 || devices[i] >= n_visible)
      return fail(TI_ERR_INVALID, "device ordinal " + std::to_string(devices[i]) + " not visible");
  if (desc->n_groups > ti::kMaxGroups) return create_chunked(desc, devices, n_devices, out);

  std::unique_ptr<ti_forest> f(new ti_forest());
  f->T = desc->n_trees;
  f->F = desc->n_features;
  f->K = desc->n_groups;
  f->LW = desc->leaf_width;
  f->accum = desc->accum_dtype;
  f->base_first = desc->base_first ? 1 : 0;
  f->lgb_zero_map = desc->lgb_zero_map ? 1 : 0;
  f->transform = desc->transform;
  f->tparam = desc->transform_param;
  f->divisor = desc->average_divisor;
  for (int k = 0; k < f->K; ++k) f->base[k] = desc->base_margin[k];
  for (int64_t i = 0; i < desc->n_nodes; ++i)
    if (desc->feature[i] >= 0) {
      if (desc->flags[i] & TI_NODE_CATEGORICAL) f->has_cat = 1;
      else if (desc->flags[i] & TI_NODE_ZERO_FLIP) f->zero_rule = 1;
    }
  f->h_group.assign(f->T, 0);
  if (f->LW == 1)
    for (int t = 0; t < f->T; ++t) f->h_group[t] = desc->tree_group[t];
  f->depth = *std::max_element(depth.begin(), depth.end());

  const size_t acc_sz = f->accum == TI_F64 ? 8 : 4;
  const int D = f->depth;
  // layout: binned heap for depth <= 8, the record layouts (6-9) for deeper
  // trees, the float explicit kernel for categorical splits;
  // TI_FORCE_LAYOUT=heap|explicit|rexplicit|lexplicit|hexplicit|texplicit
  // overrides (tests run every layout on the same forest)
  const char* force = env_knob("TI_FORCE_LAYOUT");
  std::string want = force ? force : "";
  bool use_heap = D <= kMaxHeapDepth;
  if (want == "heap" && D <= kMaxHeapDepth) use_heap = true;
  if (want == "explicit" || want == "rexplicit" || want == "lexplicit" || want == "hexplicit" ||
      want == "texplicit")
    use_heap = false;
  // categorical splits are evaluated by the explicit kernel only
  if (f->has_cat) use_heap = false;
  // binned heap (rank-binned features, 4-byte nodes) for complete-able trees
  // without LightGBM zero-missing or categorical splits; TI_FORCE_LAYOUT=heap
  // keeps the float-compare heap kernel
  bool use_bheap = use_heap && want != "heap" && f->zero_rule == 0 && D >= 1;
  if (use_bheap) {
    bool ok;
    if (f->accum == TI_F64)
      ok = pack_bheap<float, double>(desc, D, &f->bh[0], &f->h_heap_leaf_ids) &&
           pack_bheap<double, double>(desc, D, &f->bh[1], nullptr);
    else
      ok = pack_bheap<float, float>(desc, D, &f->bh[0], &f->h_heap_leaf_ids) &&
           pack_bheap<double, float>(desc, D, &f->bh[1], nullptr);
    if (!ok) {
      use_bheap = false;
      for (auto& bi : f->bh) bi = ti_forest::BinImage();
    }
  }
  if (use_bheap) {
    f->layout = 3;
  } else if (use_heap) {
    const int NI = (1 << D) - 1, NL = 1 << D;
    f->layout = 0;
    f->stride32 = static_cast<int64_t>(align16(sizeof(HeapNode<float>) * NI + acc_sz * NL * f->LW));
    f->stride64 = static_cast<int64_t>(align16(sizeof(HeapNode<double>) * NI + acc_sz * NL * f->LW));
    const int want = env_int("TI_HEAP_ROWS", 0);
    f->rows32 = pick_rows(f->F, 4, want);
    f->rows64 = pick_rows(f->F, 8, want);
    // feature byte offset: column of the [F][R] LDS image, or of the row in HBM
    const uint32_t sc32 = f->rows32 ? static_cast<uint32_t>(f->rows32) * 4u : 4u;
    const uint32_t sc64 = f->rows64 ? static_cast<uint32_t>(f->rows64) * 8u : 8u;
    if (static_cast<uint64_t>(f->F) * std::max(sc32, sc64) > ti::kMetaFeatMask)
      return fail(TI_ERR_UNSUPPORTED, "feature image offsets exceed 24 bits");
    if (f->accum == TI_F64) {
      pack_heap<float, double>(desc, D, f->stride32, sc32, &f->h_heap32, &f->h_heap_leaf_ids);
      pack_heap<double, double>(desc, D, f->stride64, sc64, &f->h_heap64, nullptr);
    } else {
      pack_heap<float, float>(desc, D, f->stride32, sc32, &f->h_heap32, &f->h_heap_leaf_ids);
      pack_heap<double, float>(desc, D, f->stride64, sc64, &f->h_heap64, nullptr);
    }
  } else {
    f->layout = 1;
    if (f->accum == TI_F64)
      pack_explicit<double>(desc, f.get(), false);
    else
      pack_explicit<float>(desc, f.get(), false);
    // record explicit slots (layout 6) unless a categorical split needs raw
    // values or another explicit kernel is forced
    bool rx_ok = false;
    if (!f->has_cat && want != "explicit") {
      std::vector<uint32_t> slot_of;
      rx_ok = plan_rx_slots(desc, f.get(), &slot_of);
      auto pack_views = [&](bool b8) {
        if (f->accum == TI_F64)
          return pack_rexplicit<float, double>(desc, f.get(), slot_of, &f->rx[0], b8) &&
                 pack_rexplicit<double, double>(desc, f.get(), slot_of, &f->rx[1], b8);
        return pack_rexplicit<float, float>(desc, f.get(), slot_of, &f->rx[0], b8) &&
               pack_rexplicit<double, float>(desc, f.get(), slot_of, &f->rx[1], b8);
      };
      // u8 bins where every feature's thresholds fit them and layout 9 takes
      // the forest (only layout 9 reads u8 images; TI_RX_B8=0 keeps u16)
      const bool try8 = rx_ok && env_int("TI_RX_B8", 1) != 0 &&
                        (want.empty() || want == "texplicit");
      bool b8 = try8 && pack_views(true) &&
                (plan_tx8(desc, f.get(), slot_of, D) || plan_tx(desc, f.get(), slot_of, D));
      if (!b8 && rx_ok) rx_ok = pack_views(false);
      if (rx_ok) {
        f->layout = 6;
        // trees in flight per lane: 16 for shallow-on-average forests (C3,
        // mean leaf depth ~9: 7.70 ms vs 7.79 at 8), 8 for deep ones (C4,
        // sklearn depth 16: 3.06 ms vs 3.13 at 16); profiles/r2_rx_sweep.jsonl
        const double md = mean_leaf_depth(desc);
        f->rx_ilp = md < 12.0 ? 16 : 8;
        const int force_ilp = env_int("TI_RX_ILP", 0);
        if (force_ilp > 0) f->rx_ilp = force_ilp >= 16 ? 16 : force_ilp >= 8 ? 8 : 4;
        // small trees: a heap top and the rest staged in LDS (layout 9; C3
        // 1M rows 5.83 vs 6.15 ms for layout 7), or all records staged
        // (layout 7, forced, or when layout 9 does not fit); deep trees too large for a
        // stage: heap tops in LDS, the rest gathered (layout 8)
        const bool auto_ok = want != "rexplicit" && want != "hexplicit" && want != "lexplicit";
        if (b8) {
          f->layout = 9;   // u8 bins (planned above)
        } else if ((want == "texplicit" || auto_ok) &&
                   (plan_tx8(desc, f.get(), slot_of, D, true) || plan_tx(desc, f.get(), slot_of, D))) {
          // layout 9 (the compact u16 bottom where it fits, else records)
        } else if ((want == "lexplicit" || auto_ok) &&
                   plan_lx_stages(f.get(), f->T)) {
          f->layout = 7;
        } else if (want == "hexplicit" ||
                   (want != "rexplicit" && D >= kHxMinDepth)) {
          plan_htop(desc, f.get(), slot_of, D);
        }
      } else {
        for (auto& rx : f->rx) rx = ti_forest::RecExplicit();
        f->h_rx_base.clear();
        f->h_rx_nint.clear();
        f->rx_slots = 0;
      }
    }
  }
  keep_shap_source(desc, f.get());
  for (int i = 0; i < n_devices; ++i) {
    f->devs.emplace_back(new DeviceForest());
    rc = upload_device(f.get(), *f->devs.back(), devices[i]);
    if (rc) {
      for (auto& d : f->devs) free_device(*d);
      return rc;
    }
  }
  // host images are no longer needed once every replica is resident
  f->h_heap32.clear(); f->h_heap32.shrink_to_fit();
  f->h_heap64.clear(); f->h_heap64.shrink_to_fit();
  f->h_heap_leaf_ids.clear(); f->h_heap_leaf_ids.shrink_to_fit();
  f->h_nodes.clear(); f->h_nodes.shrink_to_fit();
  f->h_thr64.clear(); f->h_thr64.shrink_to_fit();
  f->h_cat_words.clear(); f->h_cat_words.shrink_to_fit();
  f->h_leaves.clear(); f->h_leaves.shrink_to_fit();

  f->h_exp_src.clear();
  f->h_exp_src.shrink_to_fit();
  for (auto& rx : f->rx) {
    rx.recs.clear();
    rx.recs.shrink_to_fit();
    rx.tbl.clear();
    rx.tbl.shrink_to_fit();
  }
  f->h_tx8_val.clear(); f->h_tx8_val.shrink_to_fit();
  f->h_tx8_ord.clear(); f->h_tx8_ord.shrink_to_fit();
  f->h_rx_base.clear(); f->h_rx_base.shrink_to_fit();
  f->h_rx_nint.clear(); f->h_rx_nint.shrink_to_fit();
  for (auto& bi : f->bh) {
    bi.img.clear();
    bi.img.shrink_to_fit();
    bi.fix_img.clear();
    bi.fix_img.shrink_to_fit();
    bi.tbl.clear();
    bi.tbl.shrink_to_fit();
  }
  *out = f.release();
  return TI_OK;
}

int ti_forest_destroy(ti_forest* forest) {
  if (!forest) return TI_OK;
  for (auto& p : forest->parts) ti_forest_destroy(p.release());
  for (auto& d : forest->devs) free_device(*d);
  delete forest;
  return TI_OK;
}

int ti_forest_get_info(const ti_forest* f, ti_forest_info* info) {
  if (!f || !info) return fail(TI_ERR_INVALID, "null argument");
  info->layout = f->layout;
  info->depth = f->depth;
  info->n_trees = f->T;
  info->n_groups = f->K;
  info->n_features = f->F;
  const ti_forest* bf = f;
  while (!bf->parts.empty()) bf = bf->parts[0].get();
  info->n_devices = static_cast<int32_t>(bf->devs.size());
  info->device_bytes = 0;
  if (f->parts.empty()) {
    info->device_bytes = f->devs.empty() ? 0 : f->devs[0]->bytes;
  } else {
    for (auto& p : f->parts) info->device_bytes += p->devs.empty() ? 0 : p->devs[0]->bytes;
  }
  info->tree_stride_bytes = f->layout == 0 ? f->stride32 : f->layout == 3 ? f->bh[0].stride : 0;
  // walk id: the kernel variant a PMC pass was taken on (bench.py matches it)
  info->walk = bheap_fixed(f, TI_F32, TI_OUTPUT_PREDICT) ? (TI_FIX_SROOT ? 2 : 1) : 0;
  info->bin_bits = f->layout == 3 ? (f->bh[0].b16 ? 16 : 8)
                   : (f->layout >= 6 && f->layout <= 9) ? (f->rx[0].b8 ? 8 : 16) : 0;
  info->tree_ilp = f->layout == 6 ? f->rx_ilp : f->layout == 8 ? f->hx_ilp
                   : (f->layout == 7 || f->layout == 9) ? f->lx_ilp : 0;
  info->n_stages = (f->layout == 7 || f->layout == 9) && !f->h_lx_stage.empty()
                       ? static_cast<int32_t>(f->h_lx_stage.size() - 1) : 0;
  info->top_depth = (f->layout == 8 || f->layout == 9) ? f->hx_top : 0;
  info->bottom = f->layout == 9 ? f->tx8 : 0;
  // the TreeSHAP coefficient table of slot 0 (of the first part)
  const ti_forest* sf = f->parts.empty() ? f : f->parts[0].get();
  info->shap_table = sf->devs.empty() ? 0 : sf->devs[0]->shap_tab_state.load();
  info->reserved1 = 0;
  info->shap_table_bytes = info->shap_table == 1 ? sf->shap_tab_len * sf->shap_tab_mt : 0;
  info->shap_table_build_ms = sf->shap_tab_build_ms;
  return TI_OK;
}

int ti_forest_set_option(ti_forest* f, int32_t option, int64_t value) {
  if (!f) return fail(TI_ERR_INVALID, "null forest");
  for (auto& p : f->parts) {
    const int rc = ti_forest_set_option(p.get(), option, value);
    if (rc) return rc;
  }
  std::lock_guard<std::mutex> lk(f->shap_mu);
  switch (option) {
    case TI_OPT_SHAP_TABLE_ROWS:
      if (value < 0) return fail(TI_ERR_INVALID, "TI_OPT_SHAP_TABLE_ROWS must be >= 0");
      f->shap_tab_rows = value;
      return TI_OK;
    case TI_OPT_SHAP_TABLE_MB:
      if (value < 0) return fail(TI_ERR_INVALID, "TI_OPT_SHAP_TABLE_MB must be >= 0");
      f->shap_tab_mb = value;
      return TI_OK;
    case TI_OPT_HOST_REGISTER:
      if (value != 0 && value != 1) return fail(TI_ERR_INVALID, "TI_OPT_HOST_REGISTER must be 0 or 1");
      f->host_register.store(static_cast<int32_t>(value));
      return TI_OK;
    default:
      return fail(TI_ERR_INVALID, "unknown option " + std::to_string(option));
  }
}

int ti_output_shape(const ti_forest* f, int32_t kind, int64_t n_rows, int64_t* out_len,
                    int32_t* out_dtype) {
  if (!f || !out_len || !out_dtype) return fail(TI_ERR_INVALID, "null argument");
  if (kind < TI_OUTPUT_MARGIN || kind > TI_OUTPUT_CONTRIB) return fail(TI_ERR_INVALID, "bad output kind");
  if (n_rows < 0) return fail(TI_ERR_INVALID, "negative n_rows");
  *out_len = n_rows * output_width(f, kind);
  *out_dtype = output_dtype(f, kind);
  return TI_OK;
}

static int check_call(const ti_forest* f, const void* X, int32_t xdt, int64_t rows, int32_t cols,
                      int64_t stride, int32_t kind, const void* out, int64_t out_len) {
  if (!f) return fail(TI_ERR_INVALID, "null forest");
  if (xdt != TI_F32 && xdt != TI_F64) return fail(TI_ERR_INVALID, "x_dtype must be TI_F32 or TI_F64");
  if (kind < TI_OUTPUT_MARGIN || kind > TI_OUTPUT_CONTRIB) return fail(TI_ERR_INVALID, "bad output kind");
  if (rows < 0) return fail(TI_ERR_INVALID, "negative n_rows");
  if (rows == 0) return TI_OK;
  if (!X || !out) return fail(TI_ERR_INVALID, "null data pointer");
  if (cols <= 0) return fail(TI_ERR_INVALID, "n_cols must be > 0");
  if (stride < cols) return fail(TI_ERR_INVALID, "row_stride < n_cols");
  if (out_len < rows * output_width(f, kind))
    return fail(TI_ERR_INVALID, "output buffer too small: need " +
                                    std::to_string(rows * output_width(f, kind)) + " elements");
  return TI_OK;
}

int ti_predict(ti_forest* f, const void* X, int32_t xdt, int64_t rows, int32_t cols,
               int64_t stride, int32_t kind, void* out, int64_t out_len) {
  int rc = check_call(f, X, xdt, rows, cols, stride, kind, out, out_len);
  if (rc || rows == 0) return rc;
  ti_forest* bf = base_forest(f);   // a chunked forest's parts share its device list
  const int nd = static_cast<int>(bf->devs.size());
  const size_t xs = dtype_size(xdt);
  const size_t os = dtype_size(output_dtype(f, kind)) * output_width(f, kind);
  const int64_t per = (rows + nd - 1) / nd;
  const unsigned char* xb = static_cast<const unsigned char*>(X);
  unsigned char* ob = static_cast<unsigned char*>(out);
  const bool hreg = bf->host_register.load() != 0;
  if (nd == 1)
    return predict_shard(f, 0, *bf->devs[0], xb, xdt, rows, cols, stride, kind, ob, hreg ? 1 : 0);
  // registered buffers (TI_OPT_HOST_REGISTER) with several devices: the whole
  // X and output are page-locked once here, before the shard threads start,
  // and unlocked after they join (shard threads registering their
  // own page-rounded slices shared boundary pages, and one thread's unregister
  // could unlock pages under another's in-flight DMA).  If either span cannot
  // be registered every shard takes the pinned staging chunks.
  HostSpan all_x, all_o;
  int reg_mode = 0;
  if (hreg && per > chunk_rows(static_cast<size_t>(stride) * xs)) {
    const size_t x_bytes = static_cast<size_t>((rows - 1) * stride + cols) * xs;
    if (all_x.reg(xb, x_bytes, true) && all_o.reg(ob, static_cast<size_t>(rows) * os, true))
      reg_mode = 2;
  }
  std::vector<int> rcs(nd, TI_OK);
  std::vector<std::string> errs(nd);
  std::vector<std::thread> th;
  for (int i = 0; i < nd; ++i) {
    const int64_t r0 = per * i;
    const int64_t r1 = std::min(rows, r0 + per);
    if (r0 >= r1) break;
    th.emplace_back([&, i, r0, r1]() {
      rcs[i] = predict_shard(f, i, *bf->devs[i], xb + r0 * stride * xs, xdt, r1 - r0, cols, stride,
                             kind, ob + r0 * os, reg_mode);
      if (rcs[i]) errs[i] = g_last_error;
    });
  }
  for (auto& t : th) t.join();   // before all_x / all_o unregister
  for (int i = 0; i < nd; ++i)
    if (rcs[i]) return fail(rcs[i], "device slot " + std::to_string(i) + ": " + errs[i]);
  return TI_OK;
}

int ti_transform_device(ti_forest* f, int32_t slot, const void* margin, int64_t rows, void* out,
                        int64_t out_len, void* stream) {
  if (!f) return fail(TI_ERR_INVALID, "null forest");
  if (rows < 0) return fail(TI_ERR_INVALID, "negative row count");
  if (rows == 0) return TI_OK;
  if (!margin || !out) return fail(TI_ERR_INVALID, "null margin or output");
  if (margin == out) return fail(TI_ERR_INVALID, "margin and output must not alias");
  if (out_len < rows * output_width(f, TI_OUTPUT_PREDICT))
    return fail(TI_ERR_INVALID, "output buffer too small");
  ti_forest* bf = base_forest(f);
  if (slot < 0 || slot >= static_cast<int>(bf->devs.size()))
    return fail(TI_ERR_INVALID, "device_slot out of range");
  TI_HIP(hipSetDevice(bf->devs[slot]->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int threads = 256;
  const unsigned grid = static_cast<unsigned>((rows + threads - 1) / threads);
  if (f->accum == TI_F64)
    hipLaunchKernelGGL(transform_rows_kernel<double>, dim3(grid), dim3(threads), 0, s,
                       static_cast<const double*>(margin), rows, f->K, f->transform, f->tparam,
                       static_cast<double*>(out));
  else
    hipLaunchKernelGGL(transform_rows_kernel<float>, dim3(grid), dim3(threads), 0, s,
                       static_cast<const float*>(margin), rows, f->K, f->transform, f->tparam,
                       static_cast<float*>(out));
  TI_HIP(hipGetLastError());
  return TI_OK;
}

int ti_predict_device(ti_forest* f, int32_t slot, const void* X, int32_t xdt, int64_t rows,
                      int32_t cols, int64_t stride, int32_t kind, void* out, int64_t out_len,
                      void* stream) {
  int rc = check_call(f, X, xdt, rows, cols, stride, kind, out, out_len);
  if (rc || rows == 0) return rc;
  ti_forest* bf = base_forest(f);
  if (slot < 0 || slot >= static_cast<int>(bf->devs.size()))
    return fail(TI_ERR_INVALID, "device_slot out of range");
  DeviceForest& d = *bf->devs[slot];
  TI_HIP(hipSetDevice(d.device));
  return launch_any(f, slot, X, xdt, rows, cols, stride, kind, out, static_cast<hipStream_t>(stream));
}

}  // extern "C"
