/*
 * treeinfer.h — C ABI of the MI355X batched tree-ensemble inference engine
 * (libtreeinfer.so, built from kfserving_amd/csrc/).
 *
 * This is the drop-in boundary for the KFServing tree-predict hot path.
 * The reference never calls a GPU: its three tree plugins hand a batch to a
 * third-party CPU library through that library's own ctypes binding:
 *
 *   python/xgbserver/xgbserver/model.py:46-47
 *       xgb.DMatrix(request["instances"]) ; self._booster.predict(dmatrix)
 *       -> upstream xgboost 0.82 C API  XGBoosterPredict(BoosterHandle,
 *          DMatrixHandle, int option_mask, unsigned ntree_limit,
 *          bst_ulong* out_len, const float** out_result)
 *   python/lgbserver/lgbserver/model.py:46-51
 *       self._booster.predict(pd.concat(dfs))
 *       -> upstream lightgbm 2.3.1 C API  LGBM_BoosterPredictForMat(handle,
 *          const void* data, int data_type, int32 nrow, int32 ncol,
 *          int is_row_major, int predict_type, int num_iteration,
 *          const char* parameter, int64* out_len, double* out_result)
 *   python/sklearnserver/sklearnserver/model.py:46-51
 *       self._model.predict(np.array(instances))
 *       -> sklearn ForestRegressor/ForestClassifier.predict (Cython)
 *
 * and each plugin's load() builds the library handle:
 *   python/xgbserver/xgbserver/model.py:35-41   xgb.Booster(model_file=...)
 *   python/lgbserver/lgbserver/model.py:36-42   lgb.Booster(model_file=...)
 *   python/sklearnserver/sklearnserver/model.py:32-41  joblib.load(...)
 *
 * The entry points below replace those library calls one for one, keeping
 * the conventions of the libraries' own C APIs: int return (0 = success,
 * negative = error), a thread-local last-error string, an opaque handle
 * created from the model and released by the caller, caller-owned output
 * buffers.  Host code (the kfserving_amd package) parses the model files itself
 * into the canonical structure-of-arrays forest described by
 * ti_forest_desc and binds these symbols with ctypes.
 *
 * Canonical split semantics (one rule for all three libraries):
 *   at internal node n with feature f = feature[n], input value x = X[row,f]:
 *     LightGBM inputs only (desc.lgb_zero_map): |x| <= 1e-35f  ->  x = 0
 *     if x is NaN:            go left iff flags[n] & TI_NODE_NAN_LEFT
 *     else if x == 0 and (flags[n] & TI_NODE_ZERO_FLIP):
 *                             go left iff !(0 <= threshold[n])
 *     else:                   go left iff x <= threshold[n]
 *   categorical nodes (flags[n] & TI_NODE_CATEGORICAL; LightGBM
 *   Tree::CategoricalDecision, decision_type bit 0) replace all of the above:
 *     v = (int)x truncated toward zero; NaN, x <= -1 and x >= 2^31 go right
 *     (static_cast<int> yields INT_MIN there on x86, which LightGBM sends right);
 *     go left iff v / 32 < cat_nwords[n] and bit v % 32 of
 *     cat_bits[cat_offset[n] + v / 32] is set (Common::FindInBitset).
 *   The host encodes each library's rule into threshold/flags:
 *     XGBoost  (x < t, f32)  : threshold = nextafterf(t, -inf) (NaN if t=-inf),
 *                              NAN_LEFT = default_left
 *     LightGBM (x <= t, f64) : threshold = t, NAN_LEFT / ZERO_FLIP from the
 *                              node's missing type (None / Zero / NaN)
 *     sklearn  (f32 x <= f64 t): threshold = t, NAN_LEFT = missing_go_to_left
 *   For float32 inputs the library compares against round_down_f32(threshold),
 *   which is exact for every float32 x; float64 inputs compare in float64.
 */
#ifndef TREEINFER_H_
#define TREEINFER_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TI_ABI_VERSION 4

/* return codes */
#define TI_OK               0
#define TI_ERR_INVALID     -1   /* bad argument / malformed forest        */
#define TI_ERR_DEVICE      -2   /* HIP runtime error                      */
#define TI_ERR_NOMEM       -3   /* host or device allocation failed       */
#define TI_ERR_UNSUPPORTED -4   /* forest shape the engine cannot run     */

/* element types */
#define TI_F32 0
#define TI_F64 1
#define TI_I32 2

/* node flag bits (ti_forest_desc.flags) */
#define TI_NODE_NAN_LEFT   0x01  /* NaN input goes left                    */
#define TI_NODE_ZERO_FLIP  0x02  /* x == 0 takes the opposite of (0 <= t)  */
#define TI_NODE_CATEGORICAL 0x04 /* bitset membership split (LightGBM)     */

/* output transforms applied after accumulation (ti_forest_desc.transform) */
#define TI_TRANSFORM_IDENTITY    0
#define TI_TRANSFORM_SIGMOID     1  /* 1/(1+exp(-param*x)), per output       */
#define TI_TRANSFORM_SOFTMAX     2  /* over the n_groups outputs             */
#define TI_TRANSFORM_ARGMAX      3  /* index of the first maximum, as value  */
#define TI_TRANSFORM_HINGE       4  /* x > 0 ? 1 : 0                         */
#define TI_TRANSFORM_EXP         5  /* exp(x)                                */
#define TI_TRANSFORM_SIGNSQUARE  6  /* sign(x) * x * x (LightGBM sqrt)       */
#define TI_TRANSFORM_LOG1PEXP    7  /* log(1 + exp(x)) (LightGBM xentlambda) */
#define TI_TRANSFORM_STEP        8  /* x >= 0 ? 1 : 0 (sklearn binary GradientBoosting label) */

/* what ti_predict writes */
#define TI_OUTPUT_MARGIN   0  /* raw score (after base/average), [rows, K]     */
#define TI_OUTPUT_PREDICT  1  /* transformed score, [rows, K] or [rows]       */
#define TI_OUTPUT_LEAF     2  /* library leaf id per tree (int32), [rows, T]   */
#define TI_OUTPUT_CONTRIB  3  /* TreeSHAP contributions, [rows, K * (F + 1)]:  */
                              /* per group F feature columns, then the bias     */
                              /* (xgboost pred_contribs); needs desc.cover      */

/*
 * Canonical forest: host structure-of-arrays over the nodes of all trees,
 * trees concatenated.  Node indices in left/right are tree-local.
 * All pointers are read during ti_forest_create only.
 */
typedef struct ti_forest_desc {
  int32_t abi_version;        /* = TI_ABI_VERSION                                   */
  int32_t n_trees;            /* T                                                  */
  int32_t n_features;         /* F: columns the forest may read                     */
  int32_t n_groups;           /* K: outputs per row                                 */
  int32_t leaf_width;         /* 1: scalar leaf added to output tree_group[t];      */
                              /* K: vector leaf added to all K outputs              */
  int32_t accum_dtype;        /* TI_F32 (XGBoost) or TI_F64 (LightGBM, sklearn)     */
  int32_t base_first;         /* 1: acc starts at base_margin (xgboost>=1, lgb, sk) */
                              /* 0: acc starts at 0, margin = base + acc (xgb 0.82) */
  int32_t lgb_zero_map;       /* 1: |x| <= 1e-35f reads as 0 (LightGBM predictor)   */
  int64_t n_nodes;            /* N                                                  */
  const int64_t* tree_offset; /* [T+1] first node of each tree                      */
  const int32_t* tree_group;  /* [T]   output group of each tree (leaf_width == 1)  */
  const int32_t* feature;     /* [N]   split feature, -1 for a leaf                 */
  const double*  threshold;   /* [N]   canonical threshold: left iff x <= t         */
  const uint8_t* flags;       /* [N]   TI_NODE_* bits                               */
  const int32_t* left;        /* [N]   left child (tree-local), -1 for a leaf       */
  const int32_t* right;       /* [N]   right child (tree-local), -1 for a leaf      */
  const int32_t* leaf_id;     /* [N]   id reported by TI_OUTPUT_LEAF for a leaf     */
  const double*  leaf_value;  /* [N * leaf_width] leaf payload (read for leaves)    */
  const double*  base_margin; /* [K]                                                */
  double  average_divisor;    /* margin /= divisor after accumulation (1 = none)    */
  int32_t transform;          /* TI_TRANSFORM_*                                     */
  int32_t reserved0;
  double  transform_param;    /* sigmoid scale                                      */
  /* categorical splits (ABI 2); NULL / 0 when the forest has none.  Replaces
   * cat_boundaries / cat_threshold of a LightGBM tree (tree.h, model text v3). */
  int64_t n_cat_words;        /* W                                                  */
  const uint32_t* cat_bits;   /* [W]   bitset words of all categorical nodes        */
  const int64_t* cat_offset;  /* [N]   first word of node n's bitset                */
  const int32_t* cat_nwords;  /* [N]   words in node n's bitset                     */
  /* node covers (ABI 3): the child weights of TreeSHAP (xgboost sum_hess,
   * LightGBM internal/leaf counts, sklearn weighted_n_node_samples); NULL when
   * the model file has none -- TI_OUTPUT_CONTRIB is then unsupported.  Replaces
   * XGBoosterPredict(option_mask = pred_contribs) / LGBM predict_type = 3. */
  const double*  cover;       /* [N]                                                */
} ti_forest_desc;

typedef struct ti_forest ti_forest;   /* opaque, owns device memory */

/* Layout the engine chose for a forest (diagnostics, bench byte models). */
typedef struct ti_forest_info {
  int32_t layout;             /* 0 heap (complete, LDS-staged), 1 explicit nodes,
                                 3 binned heap, 6 record explicit (gathered), 7 staged
                                 records, 8 heap tops + gathered records, 9 heap tops +
                                 staged records (2, 4 and 5 were
                                 retired in round 3)                                 */
  int32_t depth;              /* heap depth D, or max depth for explicit             */
  int32_t n_trees;
  int32_t n_groups;
  int32_t n_features;
  int32_t n_devices;
  int64_t device_bytes;       /* forest bytes resident per device                   */
  int64_t tree_stride_bytes;  /* heap layout: bytes per staged tree                 */
  int32_t walk;               /* binned heap walk of float32 input: 0 indexed step
                                 (5 VALU), 1 fixed-layout step (4 VALU),
                                 2 fixed-layout step with the scalar-loaded root     */
  int32_t bin_bits;           /* 8 or 16: bin width of the float32 image (0: none)   */
  int32_t tree_ilp;           /* record layouts: trees walked at once per lane       */
  int32_t n_stages;           /* staged layouts (7, 9): LDS stages of the forest     */
  int32_t top_depth;          /* layouts 8, 9: levels of each tree's heap top        */
  int32_t bottom;             /* layout 9: 0 records, 1 compact u8 nodes (plan_tx8),
                                 2 compact u16 nodes, 3 compact u16 nodes walked two
                                 lanes a row (round 6)                              */
  /* ABI 4: the TreeSHAP coefficient table of device slot 0 */
  int32_t shap_table;         /* 1 built, 0 not (yet) built, -1 not buildable: over
                                 TI_OPT_SHAP_TABLE_MB or its allocation failed; the
                                 extend / unwind kernel serves every batch          */
  int32_t reserved1;
  int64_t shap_table_bytes;   /* device bytes of the built table                     */
  double  shap_table_build_ms;/* host wall time of the last table build             */
} ti_forest_info;

/* ti_forest_set_option options (ABI 4) */
#define TI_OPT_SHAP_TABLE_ROWS 1  /* TI_OUTPUT_CONTRIB batches of at most this many rows
                                     use the TreeSHAP coefficient table (0: never);
                                     default 16384 or $TI_SHAP_TABLE_ROWS            */
#define TI_OPT_SHAP_TABLE_MB   2  /* build the table only if it fits this many MiB per
                                     device (0: never); default 1280 or
                                     $TI_SHAP_TABLE_MB; read when a replica's table
                                     is first needed                                */
#define TI_OPT_HOST_REGISTER   3  /* 1: ti_predict page-locks the caller's X and
                                     output for a multi-chunk batch and copies
                                     straight from / to them; 0
                                     (default): pinned staging chunks.  A buffer
                                     that cannot be registered, or whose pages
                                     another registration already holds, takes
                                     the staging chunks.  The caller must not
                                     predict concurrently into buffers sharing a
                                     page with this call's.                         */

/* Upload the forest to each listed device (HIP device ordinals).  HIP is
 * initialised here, not at library load, so a process may fork before it.
 * Replaces: xgb.Booster(model_file=...) (xgbserver/model.py:38-39),
 *           lgb.Booster(model_file=...) (lgbserver/model.py:39-40),
 *           joblib.load(...)            (sklearnserver/model.py:38). */
int ti_forest_create(const ti_forest_desc* desc, const int32_t* devices,
                     int32_t n_devices, ti_forest** out);

/* Release device memory and the handle (XGBoosterFree / LGBM_BoosterFree). */
int ti_forest_destroy(ti_forest* forest);

int ti_forest_get_info(const ti_forest* forest, ti_forest_info* info);

/* Per-forest tuning that changes speed, never results (both TreeSHAP kernels
 * produce the same contributions).  0 or TI_ERR_INVALID for an unknown option
 * or a negative value.  Replaces nothing in the libraries: xgboost and
 * LightGBM have no TreeSHAP table; this is the engine's own knob (the
 * :explain route, python/kfserving/kfserving/kfserver.py:79-82). */
int ti_forest_set_option(ti_forest* forest, int32_t option, int64_t value);

/* Number of elements and element type ti_predict writes for n_rows rows. */
int ti_output_shape(const ti_forest* forest, int32_t output_kind, int64_t n_rows,
                    int64_t* out_len, int32_t* out_dtype);

/* Host-buffer predict.  X: [n_rows, n_cols] row-major with row_stride
 * elements between rows, element type x_dtype (TI_F32/TI_F64); out: caller-
 * owned host buffer of out_len elements (see ti_output_shape).  Rows are
 * sharded in contiguous blocks across the forest's devices; the call blocks
 * until the result is in `out`.  Thread-safe per handle.
 * Replaces: XGBoosterPredict (xgbserver/model.py:46-47),
 *           LGBM_BoosterPredictForMat (lgbserver/model.py:51),
 *           ForestRegressor/Classifier.predict (sklearnserver/model.py:50). */
int ti_predict(ti_forest* forest, const void* X, int32_t x_dtype, int64_t n_rows,
               int32_t n_cols, int64_t row_stride, int32_t output_kind,
               void* out, int64_t out_len);

/* Device-resident predict on one of the forest's devices (device_slot indexes
 * the devices passed to ti_forest_create).  X and out are device pointers on
 * that device; the kernels are enqueued on `hip_stream` (a hipStream_t, NULL =
 * the default stream) and the call returns without synchronising. */
int ti_predict_device(ti_forest* forest, int32_t device_slot, const void* X,
                      int32_t x_dtype, int64_t n_rows, int32_t n_cols,
                      int64_t row_stride, int32_t output_kind, void* out,
                      int64_t out_len, void* hip_stream);

/* The forest's output transform (TI_OUTPUT_PREDICT semantics) applied to
 * margins summed elsewhere: in the tree-sharded mode each rank predicts
 * TI_OUTPUT_MARGIN over its slice of the trees and the partial margins are
 * summed by an RCCL reduce (kfserving_amd/tree_shard.py).  margin: [n_rows,
 * n_groups] device array of the accumulation type (base margin included);
 * out: ti_output_shape(TI_OUTPUT_PREDICT) elements on the same device, not
 * aliasing margin.  Enqueued on hip_stream; returns without synchronising.
 * Replaces the objective's PredTransform that XGBoosterPredict /
 * LGBM_BoosterPredictForMat apply after summing the trees. */
int ti_transform_device(ti_forest* forest, int32_t device_slot, const void* margin,
                        int64_t n_rows, void* out, int64_t out_len, void* hip_stream);

/* Thread-local message for the last failing call on this thread
 * (XGBGetLastError / LGBM_GetLastError). */
const char* ti_last_error(void);

/* HIP device count visible to this process (initialises HIP). */
int ti_device_count(int32_t* count);

/* TI_ABI_VERSION of the loaded library. */
int32_t ti_abi_version(void);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif  /* TREEINFER_H_ */
