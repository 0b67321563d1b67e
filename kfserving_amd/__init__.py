"""MI355X-native batched tree-ensemble inference behind KFServing's
model-server API.

Layout:
  forest.py        canonical SoA forest (the C-ABI's ti_forest_desc)
  engine.py        ctypes binding of libtreeinfer.so (include/treeinfer.h)
  formats/         XGBoost / LightGBM / sklearn model loaders
  csrc/            HIP kernels + C ABI (built into lib/libtreeinfer.so)
  kfserving/       KFModel / KFServer / repository (python/kfserving mirror)
  xgbserver/ lgbserver/ sklearnserver/   the three tree plugins
  batcher/         pkg/batcher semantics (request coalescing)
"""
__version__ = "0.1.0"
