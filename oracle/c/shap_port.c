/*
 * shap_port.c -- C/OpenMP restatement of xgboost's TreeSHAP (pred_contribs).
 * TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): the CPU baseline of the
 * GPU contributions (TI_OUTPUT_CONTRIB) in scripts/bench_configs.py and a
 * second, independent check of oracle/shap_ref.py.
 *
 * Follows upstream xgboost src/tree/tree_model.cc (not vendored under
 * /root/reference; pinned version 0.82 per python/xgbserver/setup.py:37):
 * RegTree::TreeShap (the recursion over hot/cold children, unwinding a
 * feature already on the path), ExtendPath, UnwindPath, UnwoundPathSum and
 * FillNodeMeanValues; gbtree PredictContribution adds base margin to the bias.
 * Works on the canonical forest arrays (include/treeinfer.h split rule) in
 * float64 where xgboost uses float -- the GPU kernel computes in float64 too.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

#define NODE_NAN_LEFT 0x01
#define NODE_ZERO_FLIP 0x02

typedef struct {
  int32_t feature;
  double zf, of, pw;
} pelem;

typedef struct {
  const int32_t* feature;
  const double* threshold;
  const uint8_t* flags;
  const int32_t* left;
  const int32_t* right;
  const double* leaf_value; /* [N, LW] */
  const double* cover;
  int32_t LW;
  int32_t zero_map;
} forest_view;

static int goes_left(const forest_view* f, int64_t g, double x) {
  if (f->zero_map && fabs(x) <= (double)1e-35f) x = 0.0;
  if (isnan(x)) return (f->flags[g] & NODE_NAN_LEFT) != 0;
  const double t = f->threshold[g];
  int left = x <= t;
  if (x == 0.0 && (f->flags[g] & NODE_ZERO_FLIP)) left = !(0 <= t);
  return left;
}

static void extend_path(pelem* p, int d, double zf, double of, int32_t fi) {
  p[d].feature = fi;
  p[d].zf = zf;
  p[d].of = of;
  p[d].pw = d == 0 ? 1.0 : 0.0;
  for (int i = d - 1; i >= 0; --i) {
    p[i + 1].pw += of * p[i].pw * (i + 1) / (double)(d + 1);
    p[i].pw = zf * p[i].pw * (d - i) / (double)(d + 1);
  }
}

static void unwind_path(pelem* p, int d, int pi) {
  const double of = p[pi].of, zf = p[pi].zf;
  double next = p[d].pw;
  for (int i = d - 1; i >= 0; --i) {
    if (of != 0) {
      const double tmp = p[i].pw;
      p[i].pw = next * (d + 1) / ((i + 1) * of);
      next = tmp - p[i].pw * zf * (d - i) / (double)(d + 1);
    } else {
      p[i].pw = (p[i].pw * (d + 1)) / (zf * (d - i));
    }
  }
  for (int i = pi; i < d; ++i) {
    p[i].feature = p[i + 1].feature;
    p[i].zf = p[i + 1].zf;
    p[i].of = p[i + 1].of;
  }
}

static double unwound_sum(const pelem* p, int d, int pi) {
  const double of = p[pi].of, zf = p[pi].zf;
  double next = p[d].pw, total = 0;
  for (int i = d - 1; i >= 0; --i) {
    if (of != 0) {
      const double tmp = next * (d + 1) / ((i + 1) * of);
      total += tmp;
      next = p[i].pw - tmp * zf * (d - i) / (double)(d + 1);
    } else {
      total += (p[i].pw / zf) / ((d - i) / (double)(d + 1));
    }
  }
  return total;
}

/* phi: [F + 1, LW] feature-major accumulator for one row */
static void tree_shap(const forest_view* f, int64_t b, int32_t v, const double* x, int32_t cols,
                      double* phi, pelem* parent, int d, double pz, double po, int32_t pfi) {
  pelem* path = parent + d;  /* this level's copy lives after the parent's */
  if (d > 0) memcpy(path, parent, sizeof(pelem) * (size_t)d);
  extend_path(path, d, pz, po, pfi);
  const int64_t g = b + v;
  if (f->feature[g] < 0) {
    for (int i = 1; i <= d; ++i) {
      const double w = unwound_sum(path, d, i);
      const double s = w * (path[i].of - path[i].zf);
      for (int k = 0; k < f->LW; ++k)
        phi[(size_t)path[i].feature * f->LW + k] += s * f->leaf_value[g * f->LW + k];
    }
    return;
  }
  const int32_t fe = f->feature[g];
  const double xv = fe < cols ? x[fe] : NAN;
  const int32_t l = f->left[g], r = f->right[g];
  const int32_t hot = goes_left(f, g, xv) ? l : r, cold = hot == l ? r : l;
  const double w = f->cover[g];
  const double hz = f->cover[b + hot] / w, cz = f->cover[b + cold] / w;
  double iz = 1, io = 1;
  int k = 0;
  for (; k <= d; ++k)
    if (path[k].feature == fe) break;
  if (k <= d) {
    iz = path[k].zf;
    io = path[k].of;
    unwind_path(path, d, k);
    d -= 1;
  }
  tree_shap(f, b, hot, x, cols, phi, path, d + 1, hz * iz, io, fe);
  tree_shap(f, b, cold, x, cols, phi, path, d + 1, cz * iz, 0.0, fe);
}

static void mean_values(const forest_view* f, int64_t b, int32_t v, double* mv) {
  const int64_t g = b + v;
  if (f->feature[g] < 0) {
    for (int k = 0; k < f->LW; ++k) mv[v * f->LW + k] = f->leaf_value[g * f->LW + k];
    return;
  }
  const int32_t l = f->left[g], r = f->right[g];
  mean_values(f, b, l, mv);
  mean_values(f, b, r, mv);
  for (int k = 0; k < f->LW; ++k)
    mv[v * f->LW + k] = (mv[l * f->LW + k] * f->cover[b + l] +
                         mv[r * f->LW + k] * f->cover[b + r]) / f->cover[g];
}

/* out: [rows, K * (F + 1)] float64, bias last per group (TI_OUTPUT_CONTRIB). */
int port_tree_shap(int32_t n_trees, const int64_t* tree_offset, const int32_t* tree_group,
                   const int32_t* feature, const double* threshold, const uint8_t* flags,
                   const int32_t* left, const int32_t* right, const double* leaf_value,
                   const double* cover, int32_t leaf_width, int32_t n_groups,
                   int32_t n_features, const double* base_margin, double average_divisor,
                   int32_t zero_map, int32_t max_depth, const double* X, int64_t rows,
                   int32_t cols, double* out, int32_t nthread) {
  if (nthread > 0) omp_set_num_threads(nthread);
  forest_view f = {feature, threshold, flags, left, right, leaf_value, cover, leaf_width,
                   zero_map};
  const int K = n_groups, F = n_features, LW = leaf_width;
  const int64_t W = (int64_t)K * (F + 1);
  double* bias = (double*)calloc((size_t)K, sizeof(double));
  if (!bias) return -1;
  for (int k = 0; k < K; ++k) bias[k] = base_margin[k] * average_divisor;
  int64_t max_nodes = 0;
  for (int t = 0; t < n_trees; ++t)
    if (tree_offset[t + 1] - tree_offset[t] > max_nodes) max_nodes = tree_offset[t + 1] - tree_offset[t];
  double* mv = (double*)malloc(sizeof(double) * (size_t)(max_nodes * LW));
  if (!mv) { free(bias); return -1; }
  for (int t = 0; t < n_trees; ++t) {
    mean_values(&f, tree_offset[t], 0, mv);
    if (LW == 1) bias[tree_group[t]] += mv[0];
    else for (int k = 0; k < K; ++k) bias[k] += mv[k];
  }
  free(mv);
  int rc = 0;
  const size_t path_elems = (size_t)(max_depth + 2) * (max_depth + 3) / 2 + 8;
#pragma omp parallel
  {
    pelem* paths = (pelem*)malloc(sizeof(pelem) * path_elems * 2);
    double* phi = (double*)malloc(sizeof(double) * (size_t)(F + 1) * LW);
    if (!paths || !phi) rc = -1;
#pragma omp for schedule(dynamic, 64)
    for (int64_t r = 0; r < rows; ++r) {
      if (!paths || !phi) continue;
      double* o = out + r * W;
      memset(o, 0, sizeof(double) * (size_t)W);
      for (int t = 0; t < n_trees; ++t) {
        memset(phi, 0, sizeof(double) * (size_t)(F + 1) * LW);
        tree_shap(&f, tree_offset[t], 0, X + r * cols, cols, phi, paths, 0, 1.0, 1.0, -1);
        for (int j = 0; j < F; ++j) {
          if (LW == 1) o[(int64_t)tree_group[t] * (F + 1) + j] += phi[j];
          else for (int k = 0; k < K; ++k) o[(int64_t)k * (F + 1) + j] += phi[j * LW + k];
        }
      }
      for (int k = 0; k < K; ++k) {
        for (int j = 0; j < F; ++j) o[(int64_t)k * (F + 1) + j] /= average_divisor;
        o[(int64_t)k * (F + 1) + F] = bias[k] / average_divisor;
      }
    }
    free(paths);
    free(phi);
  }
  free(bias);
  return rc;
}
