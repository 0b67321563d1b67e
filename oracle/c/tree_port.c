/*
 * tree_port.c -- C/OpenMP restatement of the three libraries' CPU predict
 * loops.  TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): it is the CPU
 * baseline bench.py times (kind "port": xgboost/lightgbm are not installed in
 * this image) and a cross-check of the numpy restatements.
 *
 * port_xgb_predict   xgboost 0.82 CPUPredictor::PredLoopSpecalize/PredValue +
 *                    RegTree::GetNext (called from python/xgbserver/xgbserver/
 *                    model.py:46-47): per row an FVec with missing flags,
 *                    per group psum = 0.0f, psum += leaf in tree order,
 *                    preds = base_margin + psum, then the objective transform.
 * port_lgb_predict   lightgbm 2.3.1 GBDT::PredictRaw + Tree::NumericalDecision
 *                    (python/lgbserver/lgbserver/model.py:51).
 * port_sk_predict    sklearn 1.7.2 _apply_dense + forest averaging
 *                    (python/sklearnserver/sklearnserver/model.py:50).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

#define XGB_TRANSFORM_NONE 0
#define XGB_TRANSFORM_SIGMOID 1

int port_num_threads(void) { return omp_get_max_threads(); }

int port_xgb_predict(int32_t n_trees, const int64_t* node_offset, const int32_t* cleft,
                     const int32_t* cright, const uint32_t* sindex, const float* value,
                     const int32_t* tree_info, int32_t n_groups, float base_margin,
                     int32_t n_features, const float* X, int64_t rows, int32_t cols,
                     int32_t transform, float* out, int32_t nthread) {
  if (nthread > 0) omp_set_num_threads(nthread);
  int rc = 0;
#pragma omp parallel
  {
    float* fv = (float*)malloc(sizeof(float) * (size_t)n_features);
    unsigned char* missing = (unsigned char*)malloc((size_t)n_features);
    if (!fv || !missing) rc = -1;
#pragma omp for schedule(static)
    for (int64_t r = 0; r < rows; ++r) {
      if (!fv || !missing) continue;
      const float* x = X + r * cols;
      /* FVec::Fill: dense numpy input, NaN = missing */
      for (int32_t f = 0; f < n_features; ++f) {
        float v = f < cols ? x[f] : NAN;
        fv[f] = v;
        missing[f] = isnan(v) ? 1 : 0;
      }
      for (int32_t g = 0; g < n_groups; ++g) {
        float psum = 0.0f;
        for (int32_t t = 0; t < n_trees; ++t) {
          if (tree_info[t] != g) continue;
          const int64_t b = node_offset[t];
          int32_t nid = 0;
          while (cleft[b + nid] != -1) {
            const uint32_t si = sindex[b + nid];
            const uint32_t f = si & 0x7fffffffu;
            if (missing[f]) {
              nid = (si >> 31) ? cleft[b + nid] : cright[b + nid];
            } else {
              nid = fv[f] < value[b + nid] ? cleft[b + nid] : cright[b + nid];
            }
          }
          psum += value[b + nid];
        }
        float m = base_margin + psum;
        if (transform == XGB_TRANSFORM_SIGMOID) m = 1.0f / (1.0f + expf(-m));
        out[r * n_groups + g] = m;
      }
    }
    free(fv);
    free(missing);
  }
  return rc;
}

static const double kZeroThreshold = 1e-35f;

int port_lgb_predict(int32_t n_trees, const int64_t* node_offset, const int64_t* leaf_offset,
                     const int32_t* split_feature, const double* threshold,
                     const int8_t* decision_type, const int32_t* left_child,
                     const int32_t* right_child, const double* leaf_value,
                     const int32_t* num_leaves, int32_t n_groups, int32_t n_features,
                     const double* X, int64_t rows, int32_t cols, double* out_raw,
                     int32_t nthread) {
  if (nthread > 0) omp_set_num_threads(nthread);
  int rc = 0;
#pragma omp parallel
  {
    double* fv = (double*)malloc(sizeof(double) * (size_t)n_features);
    if (!fv) rc = -1;
#pragma omp for schedule(static)
    for (int64_t r = 0; r < rows; ++r) {
      if (!fv) continue;
      const double* x = X + r * cols;
      for (int32_t f = 0; f < n_features; ++f) {
        double v = f < cols ? x[f] : 0.0;
        fv[f] = (fabs(v) > kZeroThreshold || isnan(v)) ? v : 0.0;
      }
      double* o = out_raw + r * n_groups;
      for (int32_t k = 0; k < n_groups; ++k) o[k] = 0.0;
      for (int32_t t = 0; t < n_trees; ++t) {
        const int64_t b = node_offset[t];
        int32_t leaf = 0;
        if (num_leaves[t] > 1) {
          int32_t node = 0;
          while (node >= 0) {
            double fval = fv[split_feature[b + node]];
            const int8_t dt = decision_type[b + node];
            const int mt = (dt >> 2) & 3;
            if (isnan(fval) && mt != 2) fval = 0.0;
            if ((mt == 1 && fval >= -kZeroThreshold && fval <= kZeroThreshold) ||
                (mt == 2 && isnan(fval))) {
              node = (dt & 2) ? left_child[b + node] : right_child[b + node];
            } else {
              node = fval <= threshold[b + node] ? left_child[b + node] : right_child[b + node];
            }
          }
          leaf = ~node;
        }
        o[t % n_groups] += leaf_value[leaf_offset[t] + leaf];
      }
    }
    free(fv);
  }
  return rc;
}

int port_sk_predict(int32_t n_trees, const int64_t* node_offset, const int32_t* children_left,
                    const int32_t* children_right, const int32_t* feature,
                    const double* threshold, const uint8_t* missing_go_to_left,
                    const double* value, int32_t value_width, int32_t n_features,
                    const float* X, int64_t rows, int32_t cols, double* out, int32_t divide,
                    int32_t nthread) {
  (void)n_features;
  if (nthread > 0) omp_set_num_threads(nthread);
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < rows; ++r) {
    const float* x = X + r * cols;
    double* o = out + r * value_width;
    for (int32_t k = 0; k < value_width; ++k) o[k] = 0.0;
    for (int32_t t = 0; t < n_trees; ++t) {
      const int64_t b = node_offset[t];
      int32_t node = 0;
      while (children_left[b + node] != -1) {
        const float v = x[feature[b + node]];
        int go_left;
        if (isnan(v))
          go_left = missing_go_to_left[b + node] != 0;
        else
          go_left = (double)v <= threshold[b + node];
        node = go_left ? children_left[b + node] : children_right[b + node];
      }
      const double* lv = value + (b + node) * value_width;
      for (int32_t k = 0; k < value_width; ++k) o[k] += lv[k];
    }
    if (divide)
      for (int32_t k = 0; k < value_width; ++k) o[k] /= n_trees;
  }
  return 0;
}
