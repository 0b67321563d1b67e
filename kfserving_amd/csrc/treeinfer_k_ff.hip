// Kernel instantiations for input type float, accumulator type float.
#include "treeinfer_dispatch.h"

namespace ti {
KernelFn kernels_ff(int layout, int K, bool fl, bool z, bool b16, int pf) {
  return select_types<float, float>(layout, K, fl, z, b16, pf);
}
}  // namespace ti
