// Kernel instantiations for input type float, accumulator type double.
#include "treeinfer_dispatch.h"

namespace ti {
KernelFn kernels_fd(int layout, int K, bool fl, bool z, bool b16, int pf) {
  return select_types<float, double>(layout, K, fl, z, b16, pf);
}
}  // namespace ti
