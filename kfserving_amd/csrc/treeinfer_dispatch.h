// treeinfer_dispatch.h — kernel selection across the per-type translation
// units.  Each treeinfer_k_<x><a>.hip instantiates every kernel of one
// (input type, accumulator type) pair, so the four compile in parallel.
#pragma once

#include "treeinfer_kernels.h"

namespace ti {

using KernelFn = void (*)(KArgs);

// layout: 0 heap, 1 explicit, 3 binned heap, 6 record explicit, 7 staged
// record explicit, 8 heap top + record bottom, 9 heap top + staged record
// bottom (2, 4 and 5 were retired in round 3); 10 selects the fixed-layout
// walk of layout 3 (bheap_fix_kernel), 11 layout 9's compact u8 bottom, 12
// its compact u16 bottom, 13 the u16 bottom walked two lanes a row.
// fl: feature image in
// LDS; z: LightGBM zero rule; b16 / pf: binned heap (and layout 9) bin width
// and prefetch depth.
template <typename XT, typename ACC, int KMAX, bool B8>
KernelFn select_tx(bool z, int pf) {
  if constexpr (sizeof(ACC) == 8) {
    if (z) return pf >= 8 ? texplicit_predict_kernel<XT, ACC, KMAX, true, 8, B8>
                  : pf == 7 ? texplicit_predict_kernel<XT, ACC, KMAX, true, 7, B8>
                            : texplicit_predict_kernel<XT, ACC, KMAX, true, 4, B8>;
  }
  return pf >= 8 ? texplicit_predict_kernel<XT, ACC, KMAX, false, 8, B8>
         : pf == 7 ? texplicit_predict_kernel<XT, ACC, KMAX, false, 7, B8>
                   : texplicit_predict_kernel<XT, ACC, KMAX, false, 4, B8>;
}

template <typename XT, typename ACC, int KMAX>
KernelFn select_layout(int layout, bool fl, bool z, bool b16, int pf) {
  if (layout == 11) {   // layout 9 with the compact u8 bottom; pf carries the tree ILP
    if constexpr (sizeof(ACC) == 8) {
      if (z) return pf >= 8 ? t8explicit_predict_kernel<XT, ACC, KMAX, true, 8>
                    : pf == 7 ? t8explicit_predict_kernel<XT, ACC, KMAX, true, 7>
                              : t8explicit_predict_kernel<XT, ACC, KMAX, true, 4>;
    }
    return pf >= 8 ? t8explicit_predict_kernel<XT, ACC, KMAX, false, 8>
           : pf == 7 ? t8explicit_predict_kernel<XT, ACC, KMAX, false, 7>
                     : t8explicit_predict_kernel<XT, ACC, KMAX, false, 4>;
  }
  if (layout == 13) {   // the compact u16 bottom, two lanes a row: 4 trees a lane (8 a group)
    if constexpr (sizeof(ACC) == 8) {
      if (z) return t16split_predict_kernel<XT, ACC, KMAX, true, 4>;
    }
    return t16split_predict_kernel<XT, ACC, KMAX, false, 4>;
  }
  if (layout == 12) {   // layout 9 with the compact u16 bottom; pf carries the tree ILP
    if constexpr (sizeof(ACC) == 8) {
      if (z) return pf >= 8 ? t16explicit_predict_kernel<XT, ACC, KMAX, true, 8>
                            : t16explicit_predict_kernel<XT, ACC, KMAX, true, 4>;
    }
    return pf >= 8 ? t16explicit_predict_kernel<XT, ACC, KMAX, false, 8>
                   : t16explicit_predict_kernel<XT, ACC, KMAX, false, 4>;
  }
  if (layout == 9) {   // pf carries the tree ILP (4, 7 or 8); b16 false: u8 bins
    if (!b16) return select_tx<XT, ACC, KMAX, true>(z, pf);
    return select_tx<XT, ACC, KMAX, false>(z, pf);
  }
  if (layout == 8) {   // pf carries the tree ILP (4 or 8)
    if constexpr (sizeof(ACC) == 8) {
      if (z) return pf >= 8 ? hexplicit_predict_kernel<XT, ACC, KMAX, true, 8>
                            : hexplicit_predict_kernel<XT, ACC, KMAX, true, 4>;
    }
    return pf >= 8 ? hexplicit_predict_kernel<XT, ACC, KMAX, false, 8>
                   : hexplicit_predict_kernel<XT, ACC, KMAX, false, 4>;
  }
  if (layout == 7) {   // pf carries the tree ILP (4, 7 or 8: about a stage's trees)
    if constexpr (sizeof(ACC) == 8) {
      if (z) return pf >= 8 ? lexplicit_predict_kernel<XT, ACC, KMAX, true, 8>
                    : pf == 7 ? lexplicit_predict_kernel<XT, ACC, KMAX, true, 7>
                              : lexplicit_predict_kernel<XT, ACC, KMAX, true, 4>;
    }
    return pf >= 8 ? lexplicit_predict_kernel<XT, ACC, KMAX, false, 8>
           : pf == 7 ? lexplicit_predict_kernel<XT, ACC, KMAX, false, 7>
                     : lexplicit_predict_kernel<XT, ACC, KMAX, false, 4>;
  }
  if (layout == 6) {   // pf carries the tree ILP (4, 8 or 16)
    if constexpr (sizeof(ACC) == 8) {
      if (z) {
        if (pf >= 16) return rexplicit_predict_kernel<XT, ACC, KMAX, true, 16>;
        if (pf >= 8) return rexplicit_predict_kernel<XT, ACC, KMAX, true, 8>;
        return rexplicit_predict_kernel<XT, ACC, KMAX, true, 4>;
      }
    }
    if (pf >= 16) return rexplicit_predict_kernel<XT, ACC, KMAX, false, 16>;
    if (pf >= 8) return rexplicit_predict_kernel<XT, ACC, KMAX, false, 8>;
    return rexplicit_predict_kernel<XT, ACC, KMAX, false, 4>;
  }
  if (layout == 10) {   // binned heap, fixed layout: float X, float sums; pf carries NG
    if constexpr (sizeof(XT) == 4 && sizeof(ACC) == 4) {
      if (b16) return pf >= 2 ? bheap_fix_kernel<XT, KMAX, true, 2> : bheap_fix_kernel<XT, KMAX, true, 1>;
      return pf >= 2 ? bheap_fix_kernel<XT, KMAX, false, 2> : bheap_fix_kernel<XT, KMAX, false, 1>;
    }
    return nullptr;
  }
  if (layout == 3) {
    if (b16) return pf <= 4 ? bheap_predict_kernel<XT, ACC, KMAX, true, 4>
                            : bheap_predict_kernel<XT, ACC, KMAX, true, 8>;
    return pf <= 4 ? bheap_predict_kernel<XT, ACC, KMAX, false, 4>
                   : bheap_predict_kernel<XT, ACC, KMAX, false, 8>;
  }
  // the LightGBM zero rule exists only for float64-accumulating forests
  if constexpr (sizeof(ACC) == 8) {
    if (z) {
      if (layout == 0) return fl ? heap_predict_kernel<XT, ACC, KMAX, true, true>
                                 : heap_predict_kernel<XT, ACC, KMAX, false, true>;
      return fl ? explicit_predict_kernel<XT, ACC, KMAX, true, true>
                : explicit_predict_kernel<XT, ACC, KMAX, false, true>;
    }
  }
  if (layout == 0) return fl ? heap_predict_kernel<XT, ACC, KMAX, true, false>
                             : heap_predict_kernel<XT, ACC, KMAX, false, false>;
  return fl ? explicit_predict_kernel<XT, ACC, KMAX, true, false>
            : explicit_predict_kernel<XT, ACC, KMAX, false, false>;
}

template <typename XT, typename ACC>
KernelFn select_types(int layout, int K, bool fl, bool z, bool b16, int pf) {
  if (K == 1) return select_layout<XT, ACC, 1>(layout, fl, z, b16, pf);
  if (K <= 4) return select_layout<XT, ACC, 4>(layout, fl, z, b16, pf);
  return select_layout<XT, ACC, 16>(layout, fl, z, b16, pf);
}

KernelFn kernels_ff(int layout, int K, bool fl, bool z, bool b16, int pf);   // float X, float acc
KernelFn kernels_fd(int layout, int K, bool fl, bool z, bool b16, int pf);   // float X, double acc
KernelFn kernels_dd(int layout, int K, bool fl, bool z, bool b16, int pf);   // double X, double acc
KernelFn kernels_df(int layout, int K, bool fl, bool z, bool b16, int pf);   // double X, float acc

}  // namespace ti
