/* plk.h -- C-ABI of libplk, the MI355X (gfx950) Felsenstein-pruning engine.
 *
 * This is the drop-in boundary under the Bio++ likelihood classes.  The
 * reference (bpp-phyl) has no FFI: its hot path is a set of C++ virtuals, and
 * each entry point below replaces one of them (paths relative to
 * /root/reference/src/Bpp/Phyl/):
 *
 *   plk_set_tip_codes / plk_set_code_table
 *       DRASRTreeLikelihoodData::initLikelihoods leaf init
 *       (Likelihood/DRASRTreeLikelihoodData.cpp:160-191) with
 *       AbstractTransitionModel::getInitValue (Model/AbstractSubstitutionModel.cpp:98-112)
 *   plk_set_pattern_weights
 *       rootWeights_ (Likelihood/AbstractTreeLikelihoodData.h:91)
 *   plk_set_eigen
 *       SubstitutionModel::getEigenValues / getColumnRightEigenVectors /
 *       getRowLeftEigenVectors (Model/SubstitutionModel.h:498-525)
 *   plk_update_pmatrices
 *       AbstractHomogeneousTreeLikelihood::computeTransitionProbabilitiesForNode
 *       (Likelihood/AbstractHomogeneousTreeLikelihood.cpp:354-414) and
 *       AbstractSubstitutionModel::getPij_t / getdPij_dt / getd2Pij_dt2
 *       (Model/AbstractSubstitutionModel.cpp:426-641); NH twin
 *       Likelihood/AbstractNonHomogeneousTreeLikelihood.cpp:407-470
 *   plk_set_pmatrix
 *       closed-form getPij_t models computed on the host (T92::getPij_t,
 *       Model/Nucleotide/T92.cpp:355-386) copied into pxy_
 *   plk_update_partials
 *       RHomogeneousTreeLikelihood::computeSubtreeLikelihood
 *       (Likelihood/RHomogeneousTreeLikelihood.cpp:802-863); NH twin
 *       Likelihood/RNonHomogeneousTreeLikelihood.cpp:1286-1350
 *   plk_root_loglik
 *       RHomogeneousTreeLikelihood::getLogLikelihood / getLogLikelihoodForASite /
 *       getLikelihoodForASiteForARateClass (Likelihood/RHomogeneousTreeLikelihood.cpp:162-216);
 *       NH Likelihood/RNonHomogeneousTreeLikelihood.cpp:168-233
 *
 * Conventions
 *   - Node indices: tips are [0, n_tips), internal nodes [n_tips, n_tips + n_internal).
 *     The transition matrix of a branch is indexed by its CHILD node index.
 *   - Matrices are row-major fp64; P[c][x][y] = Prob(y at child | x at parent).
 *   - Host buffers are borrowed for the duration of the call only; device buffers
 *     are owned by the handle.  One handle per host thread.  All work is ordered
 *     on the handle's HIP stream; plk_root_loglik and plk_get_* synchronise.
 *   - Every function returns PLK_OK (0) or a negative PLK_ERR_* code; the
 *     message of the last error is available from plk_last_error().  No C++
 *     exception crosses this boundary.
 *   - There is no CPU fallback: plk_create fails with PLK_ERR_DEVICE when no
 *     gfx950 device is usable.
 */
#ifndef PLK_H
#define PLK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: plk_timing gained `evaluations` and `host_us` (a caller built against 1 must not pass
 * its smaller struct to plk_get_timing_ex) */
#define PLK_ABI_VERSION 2

enum {
  PLK_OK = 0,
  PLK_ERR_ARG = -1,         /* bad argument (index out of range, null pointer, size) */
  PLK_ERR_DEVICE = -2,      /* HIP runtime / device error or no usable GPU */
  PLK_ERR_OOM = -3,         /* device allocation failed */
  PLK_ERR_UNSUPPORTED = -4, /* state count / class count / flag not supported */
  PLK_ERR_STATE = -5,       /* call order violated (e.g. partials before P matrices) */
  PLK_ERR_BAD_CODE = -6     /* tip code outside the code table (BadIntException) */
};

/* plk_create flags */
enum {
  PLK_FLAG_SCALING = 1u << 0,    /* exact power-of-two per-pattern rescaling (deviation,
                                    needed where the reference underflows) */
  PLK_FLAG_NONNEG_GUARD = 1u << 1 /* homogeneous root guards: drop terms <= 0
                                    (RHomogeneousTreeLikelihood.cpp:197-198,212-213);
                                    without it the NH rule clamps l<0 -> 0
                                    (RNonHomogeneousTreeLikelihood.cpp:206) */,
  PLK_FLAG_LNL_ONLY = 1u << 2,   /* 4-state fused traversal keeps interior partials in
                                    registers and materialises only fragment roots; other
                                    partials are recomputed on demand by plk_get_partials */
  PLK_FLAG_LEVELWISE = 1u << 3,  /* force one launch per tree level (every child partial
                                    re-read from HBM); for A/B measurements */
  PLK_FLAG_SUBTREE_PATTERNS = 1u << 4 /* per-subtree site-pattern compression, the reference's
                                    usePatterns = true (DRASRTreeLikelihoodData.cpp:218-332):
                                    each internal node is computed once per distinct pattern of
                                    its subtree and read through pattern links.  Links are
                                    built on the host from the tip codes and the op list (all
                                    internal children must be produced by the same call); any
                                    state count, polytomies of any degree */,
  PLK_FLAG_DOUBLE_RECURSIVE = 1u << 5 /* DRHomogeneousTreeLikelihood: keep one "upper" conditional
                                    likelihood per branch (the reference's father-side arrays,
                                    DRHomogeneousTreeLikelihood.cpp:543-651) so that
                                    plk_all_branch_derivatives serves every branch from one
                                    preorder pass; n_nodes extra partial slots in HBM */
};

/* plk_update_pmatrices deriv_mask */
enum { PLK_DERIV_P = 1u, PLK_DERIV_DP = 2u, PLK_DERIV_D2P = 4u };

/* plk_op flags */
enum { PLK_OP_ACCUMULATE = 1 /* multiply into the parent's existing partial (polytomies) */ };

/* One partial update: parent = prod_k (P_branch(child_k) . L_child_k).
 * Ops handed to one plk_update_partials call must be in postorder; the engine
 * batches consecutive independent ops into one launch. */
typedef struct plk_op {
  int32_t parent;
  int32_t n_children; /* 1..3 */
  int32_t child[3];
  int32_t flags;
} plk_op;

typedef struct plk_handle_s* plk_handle;

/* Library / device */
int plk_abi_version(void);
/* First 16 hex digits of the SHA-256 of the library's sources (the .hip and .hpp files of csrc in
 * sorted order, then this header), fixed at compile time: lets a caller check that the
 * loaded binary was built from the sources it ships with. */
const char* plk_build_id(void);
int plk_device_count(int* count);
const char* plk_last_error(plk_handle h); /* h may be NULL: last global error */

/* Create an engine instance on HIP device `device`.  (Several devices: plk_create_multi
 * below; several processes: plk_comm_init.)
 *   n_states: 2..64, n_classes: 1..16, n_patterns >= 1 (padded internally),
 *   n_models: number of eigen systems (1 for homogeneous; one per branch for NH). */
int plk_create(int device, int n_states, int n_classes, int64_t n_patterns, int n_tips, int n_internal,
               int n_models, unsigned flags, plk_handle* out);
int plk_destroy(plk_handle h);

/* Multi-GPU at the boundary (SURVEY 8(b) device_mask, 8(e)).  Site patterns are
 * independent, so a run is sharded into contiguous pattern ranges whose boundaries are
 * multiples of plk_block_size(); each device evaluates its range with no traffic during
 * the traversal, and the only exchange of an evaluation is the fixed-order block sums of
 * the root reduction, summed in global block order -- the lnL is bitwise identical for any
 * device count.
 *
 * One process, several devices: plk_create_multi takes the device list (a device may be
 * listed twice: two shards on one GPU, for tests) and the TOTAL pattern count; the handle
 * it returns accepts every call of this header with whole-alignment arguments (tip codes,
 * weights, per-pattern outputs span all patterns) and fans them out: every shard after the
 * first has a persistent host worker thread (the caller's thread runs the first), so the
 * shards' launch calls and stream waits run side by side; each device's block sums arrive in
 * mapped host memory and the caller sums them in global order (the result is needed on the
 * host, so an in-process collective would only add a hop).  Derivatives are summed over
 * shards in shard order.  Timing and plk_kernel_path report shard 0; plk_traversal_work sums
 * the shards. */
int plk_create_multi(const int* devices, int n_devices, int n_states, int n_classes, int64_t n_patterns, int n_tips,
                     int n_internal, int n_models, unsigned flags, plk_handle* out);
int plk_shard_count(plk_handle h, int* n_shards);
/* Fan-out of a multi-device handle's plk_evaluate calls since plk_reset_timing: for each of its
 * n_shards shards (plk_shard_count), the mean offset in microseconds from the caller posting
 * the evaluation to [3i] the shard's worker starting it, [3i+1] its traversal launch call
 * returning and [3i+2] its completion wait returning; spread_us[0] / [1] = mean / max over the
 * evaluations of the last minus the first shard's traversal launch.  A single-device handle
 * reports zeros (n_shards = 1). */
int plk_get_fanout(plk_handle h, int n_shards, double* offsets_us, double* spread_us, int64_t* evaluations);

/* One process per GPU (torch.distributed / MPI launch): rank r creates its handle with
 * plk_create for ITS pattern range, one rank gets an id with plk_comm_get_id and shares
 * it (any channel), and every rank calls plk_comm_init.  From then on plk_root_loglik and
 * plk_evaluate all-gather every rank's block sums over RCCL (xGMI) on the handle's stream
 * -- one fixed-size ncclAllGather per evaluation -- and return the GLOBAL lnL on every
 * rank (block_sums / site_lnl stay per rank).  Ranks must hold consecutive pattern ranges
 * in rank order with block-aligned boundaries.  Replaces nothing in the reference (which
 * is single-threaded); it is the single reduce north_star names. */
typedef struct plk_comm_id {
  char internal[128];
} plk_comm_id;
int plk_comm_get_id(plk_comm_id* id);
int plk_comm_init(plk_handle h, int n_ranks, int rank, const plk_comm_id* id);

/* The exchange's host-side bookkeeping, the same code the communicator path runs
 * (csrc/plk_exchange.hpp); host only, no GPU needed -- for callers with their own
 * collective (MPI, gloo) and for the CPU tests.  Rank r's record is `stride` doubles:
 * its block sums, zero padding, its underflow flag (1.0 / 0.0); stride = max block
 * count + 1.  reduce: the global lnL as ONE chain of adds in rank order then block order
 * (the one-process fixed-order sum of RNonHomogeneousTreeLikelihood.cpp:168-182, bitwise
 * for any rank count) and the OR of the flags.  rank_sums: v[i] = sum over ranks in rank
 * order of gathered[r * n + i] (the derivative sums). */
int plk_exchange_stride(const int64_t* counts /* n_ranks */, int n_ranks, int64_t* stride);
int plk_exchange_pack(const double* block_sums, int64_t n_blocks, int uflow, int64_t stride,
                      double* record /* stride */);
int plk_exchange_reduce(const double* gathered /* n_ranks x stride */, const int64_t* counts, int n_ranks,
                        int64_t stride, double* lnl, int* uflow);
int plk_exchange_rank_sums(const double* gathered /* n_ranks x n */, int n_ranks, int64_t n, double* v /* n */);

/* Data */
int plk_set_code_table(plk_handle h, int n_codes, const double* code_to_vec /* n_codes x S */);
int plk_set_tip_codes(plk_handle h, int tip, const uint8_t* codes /* n_patterns */);
int plk_set_pattern_weights(plk_handle h, const double* weights /* n_patterns */);
int plk_set_category_rates(plk_handle h, const double* rates /* C */, const double* probs /* C */);
int plk_set_root_frequencies(plk_handle h, const double* pi /* S */);

/* Models and transition matrices */
int plk_set_eigen(plk_handle h, int model, const double* V /* S x S */, const double* Vinv /* S x S */,
                  const double* lambda /* S */);
/* For each i < n: branch[i] (a child node index) gets P = V_m exp(lambda_m * r_c * t_i) Vinv_m
 * for every class c, with m = model[i] (model may be NULL: model 0).  Optional
 * first/second derivatives follow the reference: dP = r_c dP/dt, d2P = r_c^2 d2P/dt2. */
int plk_update_pmatrices(plk_handle h, int n, const int32_t* branch, const int32_t* model,
                         const double* t, unsigned deriv_mask);
int plk_set_pmatrix(plk_handle h, int branch, const double* P /* C x S x S */);
int plk_get_pmatrix(plk_handle h, int branch, double* P /* C x S x S */);
/* The derivative matrices plk_update_pmatrices stored with PLK_DERIV_DP (order 1: r_c dP/dt)
 * or PLK_DERIV_D2P (order 2: r_c^2 d2P/dt2) -- the reference's getdPij_dt / getd2Pij_dt2
 * (Model/AbstractSubstitutionModel.cpp:499-641) scaled as computeTransitionProbabilitiesForNode
 * stores them (Likelihood/AbstractHomogeneousTreeLikelihood.cpp:375-413). */
int plk_get_dpmatrix(plk_handle h, int branch, int order, double* dP /* C x S x S */);

/* Partials */
int plk_update_partials(plk_handle h, const plk_op* ops, int n_ops);
int plk_get_partials(plk_handle h, int node, double* out /* n_patterns x C x S, reference order */);

/* Root reduction.  lnl = sum_p w_p log(sum_c prob_c sum_s pi_s L_root[p][c][s]).
 * site_lnl (nullable) receives the per-pattern log-likelihoods (n_patterns).
 * block_sums (nullable) receives the per-4096-pattern-block weighted sums in
 * pattern order (ceil(n_patterns / 4096) values): summing them in a fixed order
 * gives a result independent of how patterns are sharded across devices. */
int plk_root_loglik(plk_handle h, int root, double* lnl, double* site_lnl, double* block_sums);

/* Underflow check of an UNSCALED handle (created without PLK_FLAG_SCALING): *flag = 1 when the
 * last root reduction (plk_evaluate, plk_root_loglik, or a fused traversal's) met a site
 * likelihood below 2^-255, or <= 0, or NaN; 0 otherwise.  Call it after the evaluation
 * returned (plk_evaluate and plk_root_loglik synchronise).  A 0 proves that a handle with
 * PLK_FLAG_SCALING would have returned bitwise the same lnL: partials are <= 1 and every
 * node's joint maximum over (class, state) is <= each of its children's (P rows sum to 1), and
 * a site's likelihood is <= its root's joint maximum, so every node's maximum was >= 2^-255
 * (one bit of rounding margin above the 2^-256 rescaling threshold) and no rescale would have
 * fired.  The Bio++ mirror evaluates unscaled first and falls back to a scaled handle only when
 * the flag is set.  Under a communicator the flag is global (every rank's, carried in the
 * block-sum all-gather), so all ranks take the same fallback decision.  PLK_ERR_STATE on a
 * scaled handle.  Replaces nothing in the reference, which has no scaling. */
int plk_root_underflow(plk_handle h, int* flag);

/* Diagnostic (PLK_DEBUG_CLOCK=1 when the traversal kernel is generated): every jit_tree4
 * workgroup stamps the shader clock counter and the constant 100 MHz counter at its start and
 * end, and each evaluation leaves one record of 5 doubles: the shader clock in MHz over all
 * workgroups, the slowest and fastest workgroup's MHz, the traversal's first-start-to-last-end
 * span in us, and the workgroup count.  *n = records held; up to cap are copied to out, and
 * the held records are cleared when all fit.  Replaces nothing in the reference. */
int plk_clock_records(plk_handle h, double* out /* cap x 5 */, int cap, int* n);

/* One likelihood evaluation as RHomogeneousTreeLikelihood::fireParameterChanged does it
 * (Likelihood/RHomogeneousTreeLikelihood.cpp:255-283): P(t) of the listed branches
 * (plk_update_pmatrices, P only), the postorder traversal (plk_update_partials) and the
 * root reduction (plk_root_loglik without per-site output), in one call. */
int plk_evaluate(plk_handle h, int n, const int32_t* branch, const int32_t* model, const double* t,
                 const plk_op* ops, int n_ops, int root, double* lnl, double* block_sums);

/* First and second derivatives of lnL with respect to the length of `branch` (a child
 * node index) for the tree of the last plk_update_partials call:
 *   d1 = d lnL / dt,  d2 = d2 lnL / dt2   (the reference's getFirstOrderDerivative
 *   returns -d1, RHomogeneousTreeLikelihood.cpp:346-360, 596-610).
 * Requires dP and d2P of the branch (plk_update_pmatrices with PLK_DERIV_DP | PLK_DERIV_D2P).
 * Replaces computeTreeDLikelihood / computeTreeD2Likelihood (:365-541, :615-791).
 * Any state and class count: 4 states with 1, 2 or 4 classes propagate L, dL, d2L up the
 * path in registers; other shapes recompute the path with dP / d2P substituted on the
 * branch (lnL is linear in one branch's P).  PLK_ERR_UNSUPPORTED with
 * PLK_FLAG_SUBTREE_PATTERNS. */
int plk_branch_derivatives(plk_handle h, int branch, double* d1, double* d2);
int plk_block_size(void);

/* Directional derivatives for two sons a, b of the traversal's root whose lengths move
 * together, t_a + alpha s and t_b + beta s:  d1 = d lnL/ds, d2 = d2 lnL/ds2 at s = 0
 * (d2 includes the mixed term 2 alpha beta d2 lnL/(dt_a dt_b)).  The reference's root
 * reparametrisation of a rooted non-homogeneous tree (reparametrizeRoot = true,
 * Likelihood/AbstractNonHomogeneousTreeLikelihood.cpp:312-330, 377-389) uses
 *   BrLenRoot:    alpha = RootPosition, beta = 1 - RootPosition
 *   RootPosition: alpha = BrLenRoot,    beta = -BrLenRoot
 * and replaces computeTreeDLikelihood / computeTreeD2Likelihood for those two variables
 * (Likelihood/RNonHomogeneousTreeLikelihood.cpp:391-560, 862-1100).  Requires dP and d2P of
 * both branches.  Any state and class count.
 * Under an RCCL communicator (plk_comm_init) this, plk_branch_derivatives and
 * plk_all_branch_derivatives return GLOBAL values on every rank: each rank's d1 and d2 are
 * all-gathered (one fixed-size ncclAllGather on the handle's stream) and summed in rank
 * order, so every rank holds the same doubles.  A multi-device handle (plk_create_multi)
 * returns the sum over its devices in shard order. */
int plk_root_pair_derivatives(plk_handle h, int a, int b, double alpha, double beta, double* d1, double* d2);

/* Double-recursive derivatives (handle created with PLK_FLAG_DOUBLE_RECURSIVE): d lnL/dt and
 * d2 lnL/dt2 for EVERY branch of the last plk_update_partials tree, written to d1[node] and
 * d2[node] (n_nodes entries each, 0 at the root).  One preorder pass computes each branch's
 * upper vector U_v (everything outside v's subtree, conditional on the state at v's father,
 * root frequencies folded in), then per branch and pattern
 *   l = sum_c p_c sum_y U_v[c][y] (P_v L_v)[c][y],  l' and l'' with r_c dP_v and r_c^2 d2P_v,
 *   d1 += w l'/l,  d2 += w (l''/l - (l'/l)^2).
 * Replaces DRHomogeneousTreeLikelihood::computeSubtreeLikelihoodPrefix (:543-651),
 * computeTreeDLikelihoodAtNode / computeTreeDLikelihoods (:287-338) and the D2 twins
 * (:373-423).  Requires dP and d2P of every branch.  Any state count the partial kernels
 * support; not with PLK_FLAG_SUBTREE_PATTERNS. */
int plk_all_branch_derivatives(plk_handle h, double* d1, double* d2);

/* Instrumentation: HIP-event timing on the handle's stream of the kernels selected
 * by the mask given to plk_set_timing (0 = off).  Each timed launch adds an event
 * pair to the stream, so time only what is needed. */
enum { PLK_TIME_PARTIALS = 1u, PLK_TIME_PMAT = 2u, PLK_TIME_ROOT = 4u, PLK_TIME_TABLES = 8u };
int plk_set_timing(plk_handle h, int mask);
/* n_launches: partials launches issued while PLK_TIME_PARTIALS was set (the timed ones) */
int plk_get_timing(plk_handle h, int64_t* n_launches, double* partials_ms, double* pmat_ms, double* root_ms);
/* All timers: PLK_TIME_TABLES times the per-traversal table builds that feed a fused
 * traversal (the 20/64-state cherry contribution tables, cherry_table_kernel), which
 * belong to the traversal's cost but are separate launches. */
typedef struct plk_timing {
  int64_t partials_launches;  /* traversal launches timed */
  double partials_ms, pmat_ms, root_ms, tables_ms;
  int64_t table_launches;     /* table-build launches timed */
  /* host side of plk_evaluate (single-device handles, always on): evaluations counted and
   * the summed wall time in microseconds of its segments -- [0] the P(t) launch call,
   * [1] the traversal launch call, [2] the block-sum launch call, [3] the completion wait,
   * [4] the host sum, [5] the caller's time between the end of one plk_evaluate and the
   * start of the next */
  int64_t evaluations;
  double host_us[6];
} plk_timing;
int plk_get_timing_ex(plk_handle h, plk_timing* out);
int plk_reset_timing(plk_handle h);
int plk_synchronize(plk_handle h);

/* Name of the kernel that served the last plk_update_partials call ("jit_tree4",
 * "tree4", "treeS", "treeM" or "levelwise"); "" before the first call. */
const char* plk_kernel_path(plk_handle h);

/* Work of the last traversal, counted on the host from the program that ran (no device
 * call).  A node update is one site pattern of one internal node's partial; the
 * reference computes n_patterns x n_internal of them per traversal
 * (RHomogeneousTreeLikelihood.cpp:839-861).  Here some are table lookups instead:
 *   - cherry tables: the partial of a cherry (two tip sons) -- and, for an unstored
 *     cherry, its contribution to the parent -- is read from a row precomputed per code
 *     pair (table_rows rows per traversal);
 *   - per-subtree pattern compression: a node is computed once per distinct pattern of
 *     its subtree.
 * node_updates counts only the updates computed per pattern.  flops are fp64 operations
 * (an FMA is 2) of the traversal kernel(s) per traversal over the padded patterns:
 * useful = on live states, issued = including MFMA padding rows (20 states run
 * 32-row tiles); table_flops = the table builds (every workgroup of the fused 4-state
 * kernel forms its own tables).  exact = 1 when counted from the fused program that
 * ran, 0 for the levelwise / interpreter paths (then the algorithmic count
 * 2 C S^2 per internal child + (k - 1) C S per combine is reported). */
typedef struct plk_work {
  int64_t patterns;       /* patterns of the handle */
  int64_t node_updates;   /* computed per pattern, summed over patterns and internal nodes */
  int64_t table_nodes;    /* internal nodes served from cherry tables (per pattern) */
  int64_t table_rows;     /* cherry-table rows built per traversal (code pairs x classes x cherries) */
  double useful_flops, issued_flops, table_flops;
  int32_t exact;
  int32_t internal_nodes; /* internal nodes of the traversal */
} plk_work;
int plk_traversal_work(plk_handle h, plk_work* out);

/* With PLK_FLAG_SUBTREE_PATTERNS: the node updates the last traversal actually computed,
 * i.e. the sum over its internal nodes of their distinct subtree patterns (the
 * uncompressed traversal computes n_patterns per node). */
int plk_compressed_work(plk_handle h, int64_t* updates);

#ifdef __cplusplus
}
#endif

#endif /* PLK_H */
