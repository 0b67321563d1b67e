// Kernel instantiations for input type double, accumulator type float.
#include "treeinfer_dispatch.h"

namespace ti {
KernelFn kernels_df(int layout, int K, bool fl, bool z, bool b16, int pf) {
  return select_types<double, float>(layout, K, fl, z, b16, pf);
}
}  // namespace ti
