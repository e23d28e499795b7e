// plk.hip -- libplk: C-ABI (include/plk.h) over the gfx950 kernels in
// plk_kernels.hpp.  Host-side responsibilities: device buffers owned by the
// handle, dependency levelling of the postorder op list (independent nodes of
// one level share a launch), launch geometry, HIP-event instrumentation.
// There is deliberately no CPU fallback anywhere in this library.

#include "../../include/plk.h"
#include "plk_kernels.hpp"
#include "plk_tree4.hpp"
#include "plk_deriv.hpp"
#include "plk_mfma64.hpp"
#include "plk_treeM.hpp"
#include "plk_jit.hpp"
#include "plk_jitm.hpp"
#include "plk_dr.hpp"
#include "plk_exchange.hpp"

#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <rccl/rccl.h>

#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

using namespace plk;

extern char** environ;

namespace {
// Environment.  The library reads a handful of variables: the JIT
// cache and its diagnostics (PLK_JIT_CACHE, PLK_JIT_LOG, PLK_JIT_DUMP), one test hook
// (PLK_TEST_COMM_FAIL) and PLK_TUNE, the engine's tuning knobs as "KEY=value,KEY=value"
// (kernel shapes and the A/B kernel choices, each covered by a bitwise or oracle test).
// Reads go through a per-thread cache keyed by the name's address (names are literals of
// this file), dropped whenever the environment changed: every API entry fingerprints the
// `environ` array (its entries' addresses -- setenv / putenv / unsetenv change them).
struct EnvCache {
  uint64_t fp = 0;
  std::vector<std::pair<const char*, const char*> > kv;
  std::vector<std::pair<std::string, std::string> > tune;  // parsed PLK_TUNE
  std::vector<std::pair<const char*, const char*> > tkv;   // key address -> value (or null)
};
thread_local EnvCache g_env;

void env_refresh() {
  uint64_t x = 1469598103934665603ull ^ (uint64_t)(uintptr_t)environ;
  for (char** e = environ; e && *e; ++e) x = (x ^ (uint64_t)(uintptr_t)*e) * 1099511628211ull;
  if (x != g_env.fp) {
    g_env.fp = x;
    g_env.kv.clear();
    g_env.tkv.clear();
    g_env.tune.clear();
    if (const char* t = std::getenv("PLK_TUNE")) {
      std::string all(t);
      size_t i = 0;
      while (i < all.size()) {
        size_t j = all.find(',', i);
        if (j == std::string::npos) j = all.size();
        const std::string item = all.substr(i, j - i);
        const size_t eq = item.find('=');
        if (eq != std::string::npos && eq > 0) g_env.tune.emplace_back(item.substr(0, eq), item.substr(eq + 1));
        i = j + 1;
      }
    }
  }
}

const char* env_get(const char* name) {
  for (const auto& p : g_env.kv)
    if (p.first == name) return p.second;
  const char* v = std::getenv(name);
  g_env.kv.emplace_back(name, v);
  return v;
}

bool env_is(const char* name, char v) {
  const char* e = env_get(name);
  return e && e[0] == v;
}

// A tuning knob of PLK_TUNE (null when not given).
const char* tune_get(const char* key) {
  for (const auto& p : g_env.tkv)
    if (p.first == key) return p.second;
  const char* v = nullptr;
  for (const auto& kv : g_env.tune)
    if (kv.first == key) v = kv.second.c_str();
  g_env.tkv.emplace_back(key, v);
  return v;
}

bool tune_is(const char* key, char v) {
  const char* e = tune_get(key);
  return e && e[0] == v;
}

int tune_int(const char* key, int def, int lo, int hi);

// per host thread (like errno): the shard workers of a multi-device handle fail on their own
thread_local std::string g_last_error;

struct EventPair {
  hipEvent_t a, b;
  int kind;  // 0 partials, 1 pmat, 2 root, 3 tables
};

using clk = std::chrono::steady_clock;

inline void cpu_relax() { __builtin_ia32_pause(); }

// Host workers of a multi-device handle (plk_create_multi).  Every shard after the first has a
// persistent thread; the caller runs shard 0 itself, so all shards' launch calls and stream
// waits run side by side instead of one shard after another (one thread issuing eight
// shards' launches put the last device ~8 x 8.5 us behind the first).  A job is posted by
// bumping `seq`; a worker spins on it for kSpinIdle after its last job (an evaluation loop
// posts every ~0.2 ms, so the workers never sleep there) and then sleeps on the condition
// variable; the caller spins on `done`.  Results are per-shard slots reduced by the caller in
// shard order, so every sum keeps the single-thread order.
struct ShardPool {
  static constexpr std::chrono::milliseconds kSpinIdle{20};
  std::vector<std::thread> threads;
  std::atomic<uint64_t> seq{0};
  std::atomic<int> done{0};
  std::atomic<int> sleepers{0};
  std::atomic<bool> stop{false};
  std::mutex m;
  std::condition_variable cv;
  const std::function<int(size_t)>* job = nullptr;
  std::vector<int> rc;
  clk::time_point t_post;
  std::vector<clk::time_point> t_start;  // per shard: the job began

  explicit ShardPool(size_t n) : rc(n, 0), t_start(n) {
    for (size_t i = 1; i < n; ++i) threads.emplace_back([this, i] { worker(i); });
  }
  ~ShardPool() {
    stop.store(true);
    {
      std::lock_guard<std::mutex> lk(m);
      cv.notify_all();
    }
    for (auto& t : threads) t.join();
  }
  void worker(size_t i) {
    uint64_t seen = 0;
    for (;;) {
      uint64_t s = seq.load(std::memory_order_acquire);
      const clk::time_point t0 = clk::now();
      for (int k = 1; s == seen && !stop.load(std::memory_order_relaxed); ++k) {
        cpu_relax();
        if ((k & 255) == 0 && clk::now() - t0 > kSpinIdle) {
          // idle: sleep (sleepers and seq are seq_cst on both sides, so a post either sees
          // this sleeper and notifies under the mutex, or this check sees the post)
          std::unique_lock<std::mutex> lk(m);
          sleepers.fetch_add(1);
          cv.wait(lk, [&] { return seq.load() != seen || stop.load(); });
          sleepers.fetch_sub(1);
        }
        s = seq.load(std::memory_order_acquire);
      }
      if (stop.load()) return;
      seen = s;
      t_start[i] = clk::now();
      rc[i] = guarded(*job, i);
      done.fetch_add(1, std::memory_order_release);
    }
  }
  // A shard job runs plk_* code that can throw (std::vector growth): on a worker thread an
  // escaping exception would call std::terminate, on the caller's it would unwind while the
  // workers still use `f` -- so every job's exception becomes its error code, and run()
  // returns only after every worker has finished.
  static int guarded(const std::function<int(size_t)>& f, size_t i) {
    try {
      return f(i);
    } catch (const std::bad_alloc&) {
      return PLK_ERR_OOM;
    } catch (...) {
      return PLK_ERR_DEVICE;
    }
  }
  // f(i) for every shard i, concurrently; returns when all are done
  void run(const std::function<int(size_t)>& f) {
    job = &f;
    done.store(0, std::memory_order_relaxed);
    t_post = clk::now();
    seq.fetch_add(1);
    if (sleepers.load() > 0) {
      std::lock_guard<std::mutex> lk(m);
      cv.notify_all();
    }
    t_start[0] = clk::now();
    rc[0] = guarded(f, 0);
    const int others = (int)rc.size() - 1;
    while (done.load(std::memory_order_acquire) < others) cpu_relax();
  }
};

}  // namespace

struct plk_handle_s {
  int device = 0;
  int S = 0, C = 0, n_tips = 0, n_internal = 0, n_nodes = 0, n_models = 0;
  int64_t n_patterns = 0, n_pad = 0;
  int n_tiles = 0, n_blocks = 0;
  unsigned flags = 0;
  int n_codes = 0;          // codes in use (compact numbering, see code_map)
  int n_codes_table = 0;    // rows of the caller's code table
  // Tip codes are stored on the device in a compact numbering: the codes that occur
  // in the uploaded alignment, in order of first appearance.  The device code table
  // and the per-tip tables then hold only those rows (an alignment of A/C/G/T uses 4
  // of DNA's 15 codes), which is what lets the fused kernels keep the tip tables of a
  // whole fragment in LDS.
  std::vector<int> code_map;            // caller code -> compact code (-1: unused)
  std::vector<int> code_orig;           // compact code -> caller code
  std::vector<double> code_table_host;  // caller's table [n_codes_table][S]
  hipStream_t stream = nullptr;
  // device buffers
  double* partials = nullptr;
  int32_t* scale = nullptr;
  uint8_t* codes = nullptr;
  double* code_table = nullptr;
  double* tipP = nullptr;
  double* pmats = nullptr;
  double* dpmats = nullptr;
  double* d2pmats = nullptr;
  double* V = nullptr;
  double* Vinv = nullptr;
  double* lambda = nullptr;
  double* weights = nullptr;
  double* rates = nullptr;
  double* probs = nullptr;
  double* pi = nullptr;
  double* site_lnl = nullptr;
  double* block_sums = nullptr;
  // small staging buffers for op lists / pmatrix requests
  KOp* d_ops = nullptr;
  size_t d_ops_cap = 0;
  // pinned host staging: P(t) requests (reused once req_done has passed) and block sums
  char* h_req = nullptr;
  char* h_req_dev = nullptr;   // device address of the staging
  size_t h_req_cap = 0;
  std::vector<int32_t> req_shadow;  // branch + model arrays now in the staging (skip rewriting them)
  bool in_eval = false;        // inside plk_evaluate: the request's reader is waited for by its stream_wait
  bool req_unrecorded = false; // a staged request's reader has no req_done record (plk_evaluate)
  hipEvent_t req_done = nullptr;
  double* h_blocks = nullptr;
  int64_t slot_stride = 0;
  // state
  bool rates_set = false, pi_set = false, table_set = false;
  std::vector<char> pmat_valid;   // per node
  std::vector<char> eigen_set;    // per model
  std::vector<char> tip_table_valid;  // per tip: tipP row matches its P(t) and the code table
  std::vector<char> tip_set;
  // instrumentation
  unsigned timing = 0;  // PLK_TIME_* mask
  std::vector<EventPair> events;
  std::vector<EventPair> event_pool;
  int64_t n_launches = 0, n_table_launches = 0;
  double acc_ms[4] = {0, 0, 0, 0};
  // host side of plk_evaluate (plk_timing::host_us): segment sums, count, end of the last one
  double host_us[6] = {0, 0, 0, 0, 0, 0};
  int64_t n_evals = 0;
  std::chrono::steady_clock::time_point last_eval_end{};
  int jit_last_gx = 0;                    // workgroups per fragment of the last JIT launch
  std::vector<int> jit_frag_gx;           // workgroups per fragment of the last JIT traversal (per fragment)
  std::string last_error;
  // host copy of the op list last uploaded to d_ops (re-used when identical)
  std::vector<KOp> h_ops;
  std::vector<plk_op> last_ops;
  std::vector<int> last_level_start;
  // fused 4-state traversal (plk_tree4.hpp)
  double* wave_sums = nullptr;
  TInstr* d_prog = nullptr;
  size_t d_prog_cap = 0;
  int32_t* d_frag = nullptr;
  size_t d_frag_cap = 0;
  unsigned* d_sbctr = nullptr;          // jit_tree4 dynamic super-block counters, one per fragment,
  size_t d_sbctr_cap = 0;               // then the exit-ticket counter (all 0 between launches)
  std::vector<plk_op> prog_ops;           // op list the cached program was built from
  bool prog_materialize = false;
  bool prog_reduce = false;
  int prog_dm = 0;                        // register levels the program was cut for
  bool prog_jit = false;                  // program cut for the tree-specialised kernel
  bool prog_ciw = false;                  // ... with every class of a pattern in one wave
  int prog_tmax = 0;                      // tips per fragment the program was cut for
  int prog_nf = 0;                        // fragments of the cached program
  std::vector<std::vector<int> > prog_tiers;  // fragment ids per tier
  int prog_root = -1;                     // node whose lnL the program reduces (-1: none)
  std::vector<char> materialized;         // per internal slot: partial present in HBM
  std::vector<int> prog_mat_after;        // per internal slot after the cached program (-1 untouched)
  // last traversal (for derivative paths) and derivative buffers
  std::vector<plk_op> trav_ops;
  std::vector<char> deriv_valid;          // per node: dP and d2P present
  double* pmatsT = nullptr;               // S = 20 / 64: transposed copy for the MFMA kernels
  bool pmatsT_dirty = true;
  double* d1_sums = nullptr;
  double* d2_sums = nullptr;
  DInstr* d_dprog = nullptr;
  size_t d_dprog_cap = 0;
  bool fused_lnl_valid = false;
  int fused_lnl_root = -1;
  // tree-specialised kernel of the cached program (plk_jit.hpp); null: interpreter
  std::vector<TInstr> prog_host;
  // treeM cherry contribution tables (plk_treeM.hpp: CherryLayout): (tip a, tip b, node)
  // per T_CHERRY of the program, the device copy, and the [table | counts | codes] buffer
  std::vector<int32_t> cherry3;
  int32_t* d_cherry3 = nullptr;
  int32_t* d_cherry_tips = nullptr;
  int32_t* d_cherry_rows = nullptr;       // per cherry: the code pairs it meets (CSR, nch + 1 starts first)
  size_t cherry_rows_cap = 0;
  int cherry_rows_max = 0;                // most code pairs of any cherry
  uint8_t* d_cherry = nullptr;
  size_t cherry3_cap = 0, cherry_tips_cap = 0, cherry_cap = 0;
  bool cherry_codes_valid = false;
  std::vector<int32_t> frag_starts_host;  // fragment start offsets, tier order
  hipFunction_t jit_fn = nullptr;
  JitShape jit_shape;
  // tree-specialised 20-state kernel on v_mfma_f64_4x4x4_4b (plk_jitm.hpp); null: not compiled yet
  hipFunction_t jitm_fn = nullptr;
  JitMShape jitm_shape;
  bool prog_jitm = false;                 // program cut for jit_treeM
  JitPlan jit_plan;            // table units / events of the current program (plk_jit.hpp)
  bool jit_plan_valid = false;
  int jit_plan_U = 0, jit_plan_budget = -1;
  int jit_plan_qb = -1;                 // quad budget the plan was built with (0: none)
  bool jit_plan_cls = false;            // the plan is one class per workgroup (it has quad units)
  double* d_cls = nullptr;              // JitShape::cls: every class's root term, [C][n_pad]
  size_t d_cls_cap = 0;
  double* fused_cls_blocks = nullptr;   // the last traversal formed its block sums here (cls_blocks_kernel)
  bool cls_site_written = false;        // ... and its per-pattern lnL (only when asked for: 8 B per pattern)
  uint8_t* d_ucodes_dc = nullptr;       // JitShape::dc: [fragment][pattern][16] unit codes
  size_t ucodes_dc_cap = 0;
  bool ucodes_dc_valid = false;
  int ucodes_dc_w = 0;                  // its 16-byte words per pattern (JitShape::dcw)
  int32_t* d_units_start = nullptr;     // CSR of the plan's units per fragment (unit_codes_dc_kernel)
  size_t units_start_cap = 0;
  uint8_t* d_ucodes = nullptr;  // code row of every table unit of jit_plan (unit_codes_kernel)
  int4* d_units = nullptr;      // (ta, tb) of every unit
  size_t ucodes_cap = 0, units_cap = 0;
  bool ucodes_valid = false;    // cleared by new tip codes and by a new plan
  int jit_resident = 0;  // workgroups of jit_fn resident at once on the device
  std::string kernel_path;                // what served the last plk_update_partials
  // per-subtree pattern compression (PLK_FLAG_SUBTREE_PATTERNS)
  std::vector<std::vector<uint8_t> > tip_codes_host;  // compact codes per tip
  bool cmp_valid = false;
  bool slots_expanded = false;                        // a derivative re-ran the traversal uncompressed
  std::vector<plk_op> cmp_ops;                        // op list the links were built for
  std::vector<std::vector<int32_t> > cmp_ids;         // per internal slot: distinct id per pattern (empty: identity)
  std::vector<int64_t> cmp_D;                         // per internal slot: distinct patterns
  std::vector<int> cmp_level_start, cmp_level_maxD;
  uint32_t* d_links = nullptr;
  size_t d_links_cap = 0;
  KOpL* d_opsl = nullptr;
  KKid* d_kidsl = nullptr;  // the compressed ops' child records
  size_t d_kidsl_cap = 0;
  size_t d_opsl_cap = 0;
  int64_t cmp_work = 0;                               // sum over nodes of distinct patterns
  // tree of the traversals so far: sons per node, merged over plk_update_partials calls
  // (an incremental call lists only the ancestors of changed branches)
  std::vector<std::vector<int> > topo_kids;
  // double-recursive derivatives (PLK_FLAG_DOUBLE_RECURSIVE, plk_dr.hpp)
  int n_mats = 0;        // transition-matrix slots: nodes, kScratchMats derivative scratch, DR M_f per node
  int dr_slot0 = 0;      // partial slot of U_v = dr_slot0 + v
  DrBranch* d_drb = nullptr;
  size_t d_drb_cap = 0;
  int2* d_drm = nullptr;
  size_t d_drm_cap = 0;
  double* dr_blk = nullptr;
  size_t dr_blk_cap = 0;
  double* dr_out = nullptr;
  // multi-device handle (plk_create_multi): one shard handle per device over contiguous,
  // block-aligned pattern ranges; the parent owns no device memory
  std::vector<plk_handle> shards;
  std::vector<int64_t> shard_start;       // first pattern of each shard (+ n_patterns at the end)
  std::unique_ptr<ShardPool> pool;        // host workers of the shards (started by the first call)
  // fan-out of the multi-device evaluations since plk_reset_timing (plk_get_fanout): per shard
  // the summed offsets (us) from the caller's post to the worker's start, to its traversal
  // launch call returning and to its completion wait returning; spread of the launches
  std::vector<double> fan_us;             // [shard][3]
  double fan_spread_sum = 0.0, fan_spread_max = 0.0;
  int64_t fan_n = 0;
  // single-device handle: when the last plk_evaluate's traversal launch call and stream wait returned
  clk::time_point t_launched{}, t_waited{};
  // RCCL communicator of a sharded multi-process run (plk_comm_init): block sums all-gathered
  // on the handle's stream and summed in global order on the device
  ncclComm_t comm = nullptr;
  int comm_ranks = 0, comm_rank = 0;
  int64_t comm_stride = 0;                // doubles per rank record in the all-gather (plk_exchange.hpp)
  int comm_uflow = 0;                     // OR of every rank's underflow flag, last evaluation
  double* d_blk_local = nullptr;          // [comm_stride] this rank's record: block sums, zeros, flag
  DrPreOp* d_drpre = nullptr;             // fused DR preorder ops (dr_pre_s4_kernel)
  size_t d_drpre_cap = 0;
  double* d_blk_all = nullptr;            // [comm_ranks][comm_stride]
  int64_t* d_comm_counts = nullptr;       // block sums per rank
  // PLK_DEBUG_CLOCK: per-workgroup clock stamps of the last jit_tree4 traversal (mapped pinned,
  // 4 u64 per workgroup) and one summary record per traversal (plk_clock_records)
  unsigned long long* h_clk = nullptr;
  unsigned long long* d_clk = nullptr;
  size_t clk_cap = 0;                     // workgroups the stamp buffer holds
  size_t clk_n = 0;                       // workgroups stamped by the pending traversal
  std::vector<double> clk_rec;
  int32_t* h_uflow = nullptr;             // mapped pinned: root-reduction underflow flag (plk_root_underflow)
  int32_t* d_uflow = nullptr;             // its device address
  double* h_blk_all = nullptr;            // mapped pinned: every rank's record [comm_ranks][comm_stride]
  double* d_blk_all_map = nullptr;        // its device address
  std::vector<int64_t> comm_counts;       // block sums per rank (host copy)
  double* d_xch = nullptr;                // derivative sums exchanged under the communicator
  double* d_xch_all = nullptr;
  size_t d_xch_cap = 0, d_xch_all_cap = 0;
};

namespace {

int fail(plk_handle h, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  if (h) h->last_error = buf;
  return code;
}

#define HIPCHK(h, call)                                                                          \
  do {                                                                                           \
    hipError_t e_ = (call);                                                                      \
    if (e_ != hipSuccess) return fail((h), PLK_ERR_DEVICE, "%s: %s", #call, hipGetErrorString(e_)); \
  } while (0)

int dalloc(plk_handle h, void** p, size_t bytes) {
  if (bytes == 0) bytes = 16;
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) {
    *p = nullptr;
    return fail(h, PLK_ERR_OOM, "hipMalloc(%zu bytes) failed: %s", bytes, hipGetErrorString(e));
  }
  return PLK_OK;
}

int ensure_cap(plk_handle h, void** p, size_t* cap, size_t bytes) {
  if (*cap >= bytes) return PLK_OK;
  if (*p) {
    // the buffer may still be read by queued work
    hipStreamSynchronize(h->stream);
    hipFree(*p);
    *p = nullptr;
  }
  size_t nb = std::max(bytes, (size_t)4096);
  int rc = dalloc(h, p, nb);
  if (rc) return rc;
  *cap = nb;
  return PLK_OK;
}

// Staging of large P(t) requests (plk_update_pmatrices): mapped pinned host memory the P(t)
// kernel reads over PCIe.  (Round 4 measured device memory written by the host over the BAR,
// 3 us less per cfg5 evaluation, and removed it: a freshly created handle whose staging
// reused freed device memory had its P(t) kernel read other data than the host had written --
// a whole shard of -inf in test_multi_device_handle_bitwise[lg08] after other tests in the
// same process, with fine-grained and with uncached allocations alike; profiles/r04/ab_runs.md.)
int req_staging(plk_handle h, size_t bytes) {
  if (h->h_req_cap >= bytes) return PLK_OK;
  h->req_shadow.clear();
  if (h->h_req) HIPCHK(h, hipHostFree(h->h_req));
  h->h_req = nullptr;
  h->h_req_dev = nullptr;
  h->h_req_cap = 0;
  bytes = (bytes + 4095) & ~(size_t)4095;
  HIPCHK(h, hipHostMalloc((void**)&h->h_req, bytes, hipHostMallocMapped));
  HIPCHK(h, hipHostGetDevicePointer((void**)&h->h_req_dev, h->h_req, 0));
  h->h_req_cap = bytes;
  return PLK_OK;
}

// Completion wait of an evaluation (spin-waiting on hipStreamQuery was measured slower: it
// contends with the launch calls).
int stream_wait(plk_handle h) {
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return PLK_OK;
}

EventPair get_events(plk_handle h, int kind) {
  EventPair e;
  if (!h->event_pool.empty()) {
    e = h->event_pool.back();
    h->event_pool.pop_back();
  } else {
    hipEventCreate(&e.a);
    hipEventCreate(&e.b);
  }
  e.kind = kind;
  return e;
}

int collect_events(plk_handle h) {
  if (h->events.empty()) return PLK_OK;
  HIPCHK(h, hipStreamSynchronize(h->stream));
  for (auto& e : h->events) {
    float ms = 0.f;
    HIPCHK(h, hipEventElapsedTime(&ms, e.a, e.b));
    h->acc_ms[e.kind] += ms;
    h->event_pool.push_back(e);
  }
  h->events.clear();
  return PLK_OK;
}

// ---------------------------------------------------------------------------
// hiprtc compilation of the tree-specialised kernels (plk_jit.hpp, plk_jitm.hpp), cached
// per process by (device, generated source) -- a module is loaded into one device's
// context, so a multi-device handle compiles once and loads once per device -- and on
// disk by source hash (PLK_JIT_CACHE=<dir>, default $XDG_CACHE_HOME/plk_jit or
// ~/.cache/plk_jit; PLK_JIT_CACHE=0 disables): a cached code object is used only when its
// stored source equals the generated one.  Modules stay loaded for the life of the process.
// ---------------------------------------------------------------------------
std::mutex g_jit_mutex;
std::map<std::pair<int, std::string>, hipFunction_t> g_jit_cache;
std::map<std::string, std::vector<char> > g_jit_code;  // compiled code objects by source

std::string jit_cache_dir() {
  const char* e = env_get("PLK_JIT_CACHE");
  if (e && (e[0] == '0' || e[0] == '\0')) return std::string();
  std::string d;
  if (e) {
    d = e;
  } else if (const char* x = env_get("XDG_CACHE_HOME")) {
    d = std::string(x) + "/plk_jit";
  } else if (const char* hm = env_get("HOME")) {
    d = std::string(hm) + "/.cache/plk_jit";
  } else {
    return std::string();
  }
  // create the directory (and a missing parent) private to the user; failure = no disk cache
  const size_t slash = d.rfind('/');
  if (slash != std::string::npos && slash > 0) mkdir(d.substr(0, slash).c_str(), 0700);
  mkdir(d.c_str(), 0700);
  struct stat st;
  if (stat(d.c_str(), &st) != 0 || !S_ISDIR(st.st_mode)) return std::string();
  return d;
}

bool read_file(const std::string& path, std::vector<char>* out) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return false;
  std::fseek(f, 0, SEEK_END);
  const long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  out->resize(n > 0 ? (size_t)n : 0);
  const bool ok = n > 0 && std::fread(out->data(), 1, (size_t)n, f) == (size_t)n;
  std::fclose(f);
  return ok;
}

void write_file_atomic(const std::string& path, const char* data, size_t n) {
  const std::string tmp = path + ".tmp" + std::to_string((long)getpid());
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) return;
  bool ok = std::fwrite(data, 1, n, f) == n;
  ok = std::fclose(f) == 0 && ok;  // a full disk often shows up only here
  if (!ok || std::rename(tmp.c_str(), path.c_str()) != 0) std::remove(tmp.c_str());
}

uint64_t fnv1a64(const std::string& s) {
  uint64_t x = 1469598103934665603ull;
  for (unsigned char c : s) x = (x ^ c) * 1099511628211ull;
  return x;
}

// "<size> <fnv1a64>" of a code object (the .sum file of a disk-cache entry)
std::string code_sum(const std::vector<char>& code) {
  uint64_t x = 1469598103934665603ull;
  for (char c : code) x = (x ^ (unsigned char)c) * 1099511628211ull;
  char b[64];
  snprintf(b, sizeof(b), "%zu %016llx", code.size(), (unsigned long long)x);
  return b;
}

// Code object of `src`: from the disk cache unless `bypass_cache`, else compiled with hiprtc
// (and stored); *from_cache tells which.
int jit_compile(plk_handle h, const std::string& src, std::vector<char>* code, bool bypass_cache, bool* from_cache) {
  *from_cache = false;
  const char* opts[] = {"--offload-arch=gfx950", "-O3"};
  const bool log = env_is("PLK_JIT_LOG", '1');
  std::string dir = jit_cache_dir(), stem;
  if (!dir.empty()) {
    char hx[17];
    // the key: the source, the options, the device's full architecture name (with its
    // target features) and the hiprtc and HIP runtime versions -- a compiler or runtime update
    // or another device variant invalidates every entry
    int maj = 0, mnr = 0, rt = 0;
    hiprtcVersion(&maj, &mnr);
    hipRuntimeGetVersion(&rt);
    hipDeviceProp_t prop;
    const std::string arch = hipGetDeviceProperties(&prop, h->device) == hipSuccess ? prop.gcnArchName : "?";
    snprintf(hx, sizeof(hx), "%016llx",
             (unsigned long long)fnv1a64(src + opts[0] + opts[1] + std::to_string(maj) + "." + std::to_string(mnr) +
                                         "/" + std::to_string(rt) + "/" + arch));
    stem = dir + "/" + hx;
    std::vector<char> stored, sum;
    // an entry is used only if its stored source equals the generated one and the code
    // object's size and hash equal the ones recorded after it was written (a truncated or
    // damaged object is never handed to hipModuleLoadData, whose ELF reader can abort)
    if (!bypass_cache && read_file(stem + ".hip", &stored) && stored.size() == src.size() &&
        std::memcmp(stored.data(), src.data(), src.size()) == 0 && read_file(stem + ".co", code) &&
        read_file(stem + ".sum", &sum) && std::string(sum.begin(), sum.end()) == code_sum(*code)) {
      if (log) std::fprintf(stderr, "[plk] jit cache hit %s.co\n", stem.c_str());
      *from_cache = true;
      return PLK_OK;
    }
  }
  const auto t0 = std::chrono::steady_clock::now();
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "plk_jit.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
    return fail(h, PLK_ERR_DEVICE, "hiprtcCreateProgram failed");
  const hiprtcResult rc = hiprtcCompileProgram(prog, 2, opts);
  if (rc != HIPRTC_SUCCESS) {
    size_t n = 0;
    hiprtcGetProgramLogSize(prog, &n);
    std::string msg(n, '\0');
    if (n) hiprtcGetProgramLog(prog, &msg[0]);
    hiprtcDestroyProgram(&prog);
    return fail(h, PLK_ERR_DEVICE, "hiprtc compile of the tree kernel failed: %s", msg.substr(0, 400).c_str());
  }
  size_t n = 0;
  hiprtcGetCodeSize(prog, &n);
  code->resize(n);
  hiprtcGetCode(prog, code->data());
  hiprtcDestroyProgram(&prog);
  if (log)
    std::fprintf(stderr, "[plk] jit compiled %zu bytes of source in %.2f s\n", src.size(),
                 std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
  if (!stem.empty()) {
    write_file_atomic(stem + ".co", code->data(), code->size());
    const std::string sm = code_sum(*code);
    write_file_atomic(stem + ".sum", sm.data(), sm.size());
    write_file_atomic(stem + ".hip", src.data(), src.size());  // last: it validates the entry
  }
  return PLK_OK;
}

int jit_function(plk_handle h, const std::string& src, const char* name, hipFunction_t* out) {
  std::lock_guard<std::mutex> lock(g_jit_mutex);
  const auto key = std::make_pair(h->device, src);
  auto it = g_jit_cache.find(key);
  if (it != g_jit_cache.end()) {
    *out = it->second;
    return PLK_OK;
  }
  auto ct = g_jit_code.find(src);
  bool from_cache = false;
  if (ct == g_jit_code.end()) {
    std::vector<char> code;
    if (int rc = jit_compile(h, src, &code, false, &from_cache)) return rc;
    ct = g_jit_code.emplace(src, std::move(code)).first;
  }
  std::vector<char>& code = ct->second;
  // PLK_JIT_DUMP=<dir>: keep the generated source and code object for inspection
  // (llvm-objdump -d --mcpu=gfx950 <dir>/plk_jit_<n>.co)
  if (const char* dir = env_get("PLK_JIT_DUMP")) {
    const std::string stem = std::string(dir) + "/plk_jit_" + std::to_string(g_jit_cache.size());
    if (FILE* f = std::fopen((stem + ".hip").c_str(), "wb")) {
      std::fwrite(src.data(), 1, src.size(), f);
      std::fclose(f);
    }
    if (FILE* f = std::fopen((stem + ".co").c_str(), "wb")) {
      std::fwrite(code.data(), 1, code.size(), f);
      std::fclose(f);
    }
  }
  hipSetDevice(h->device);
  hipModule_t mod;
  auto load = [&]() {
    try {
      return hipModuleLoadData(&mod, code.data()) == hipSuccess;
    } catch (...) {
      return false;
    }
  };
  if (!load()) {
    if (!from_cache) return fail(h, PLK_ERR_DEVICE, "hipModuleLoadData of the compiled tree kernel failed");
    // a damaged disk-cache entry: recompile and overwrite it
    (void)hipGetLastError();
    if (int rc = jit_compile(h, src, &code, true, &from_cache)) return rc;
    if (!load()) return fail(h, PLK_ERR_DEVICE, "hipModuleLoadData of the recompiled tree kernel failed");
  }
  hipFunction_t fn;
  HIPCHK(h, hipModuleGetFunction(&fn, mod, name));
  g_jit_cache.emplace(key, fn);
  *out = fn;
  return PLK_OK;
}

bool s4_supported(int C) { return C == 1 || C == 2 || C == 4 || C == 8; }

// derivative scratch: partial slots (path derivatives: dL ping-pong, d2L ping-pong; root-pair
// derivatives: five substituted root products), transition matrices and tip rows
constexpr int kDerivScratch = 6;
constexpr int kScratchMats = 4;
constexpr int kScratchTips = 4;

template <bool SCALE>
void launch_s4(plk_handle h, const KOp* d_ops, int n_ops, const PartialsArgs& a) {
  dim3 grid((a.n_tiles + 3) / 4, n_ops), block(256);
  switch (h->C) {
    case 1: partials_s4_kernel<1, SCALE><<<grid, block, 0, h->stream>>>(d_ops, a); break;
    case 2: partials_s4_kernel<2, SCALE><<<grid, block, 0, h->stream>>>(d_ops, a); break;
    case 4: partials_s4_kernel<4, SCALE><<<grid, block, 0, h->stream>>>(d_ops, a); break;
    case 8: partials_s4_kernel<8, SCALE><<<grid, block, 0, h->stream>>>(d_ops, a); break;
  }
}

template <int S, int XB>
void launch_generic_S(plk_handle h, const KOp* d_ops, int n_ops, const PartialsArgs& a, size_t lds) {
  dim3 grid((a.n_tiles + 1) / 2, n_ops), block(256);
  if (h->flags & PLK_FLAG_SCALING)
    partials_generic_kernel<S, XB, true><<<grid, block, lds, h->stream>>>(d_ops, a, h->C);
  else
    partials_generic_kernel<S, XB, false><<<grid, block, lds, h->stream>>>(d_ops, a, h->C);
}

// P^T copy of every transition matrix for the MFMA kernels (A operand rows = y),
// refreshed lazily after any P(t) change.
int ensure_pmatsT(plk_handle h) {
  if (!h->pmatsT) {
    int rc = dalloc(h, (void**)&h->pmatsT, (size_t)h->n_mats * h->C * h->S * h->S * sizeof(double));
    if (rc) return rc;
    h->pmatsT_dirty = true;
  }
  if (h->pmatsT_dirty) {
    const dim3 grid(h->n_nodes + kScratchMats, h->C);  // + the derivative scratch matrices
    if (h->S == 64)
      transpose_pmats<64><<<grid, 256, 0, h->stream>>>(h->pmats, h->pmatsT, h->C);
    else if (h->S == 20)
      transpose_pmats<20><<<grid, 256, 0, h->stream>>>(h->pmats, h->pmatsT, h->C);
    else if (h->S == 4)
      transpose_pmats<4><<<grid, 256, 0, h->stream>>>(h->pmats, h->pmatsT, h->C);
    else
      return fail(h, PLK_ERR_UNSUPPORTED, "no transposed-P path for %d states", h->S);
    HIPCHK(h, hipGetLastError());
    h->pmatsT_dirty = false;
  }
  return PLK_OK;
}

int launch_generic(plk_handle h, const KOp* d_ops, int n_ops, const PartialsArgs& a) {
  const int S = h->S;
  if (S == 64) {
    // K3: fp64 MFMA, P^T staged in LDS
    int rc = ensure_pmatsT(h);
    if (rc) return rc;
    const size_t lds = (size_t)std::max(64 * kM64Ld, h->n_codes * 64) * sizeof(double);
    dim3 grid(a.n_tiles, n_ops), block(kM64Threads);
    if (h->flags & PLK_FLAG_SCALING)
      partials_mfma64_kernel<true><<<grid, block, lds, h->stream>>>(d_ops, a, h->pmatsT, h->C);
    else
      partials_mfma64_kernel<false><<<grid, block, lds, h->stream>>>(d_ops, a, h->pmatsT, h->C);
    return PLK_OK;
  }
  if (S == 20) {
    // K2: P rows through scalar loads, tip tables in LDS
    const size_t lds = 3 * (size_t)h->C * h->n_codes * S * sizeof(double);
    if (lds <= 160 * 1024) {
      dim3 grid((a.n_tiles + 1) / 2, n_ops), block(256);
      if (h->flags & PLK_FLAG_SCALING)
        partials_sgpr_kernel<20, true><<<grid, block, lds, h->stream>>>(d_ops, a, h->pmats, h->C);
      else
        partials_sgpr_kernel<20, false><<<grid, block, lds, h->stream>>>(d_ops, a, h->pmats, h->C);
      return PLK_OK;
    }
  }
  const size_t per = (size_t)h->C * S * std::max(S, h->n_codes);
  const size_t lds = 3 * per * sizeof(double);
  if (lds > 160 * 1024) return fail(h, PLK_ERR_UNSUPPORTED, "LDS image of %zu bytes exceeds 160 KiB", lds);
  switch (S) {
    case 2: launch_generic_S<2, 2>(h, d_ops, n_ops, a, lds); break;
    case 3: launch_generic_S<3, 3>(h, d_ops, n_ops, a, lds); break;
    case 4: launch_generic_S<4, 4>(h, d_ops, n_ops, a, lds); break;
    case 20: launch_generic_S<20, 20>(h, d_ops, n_ops, a, lds); break;
    default: return fail(h, PLK_ERR_UNSUPPORTED, "state count %d has no kernel instance", S);
  }
  return PLK_OK;
}

int refresh_tip_tables(plk_handle h) {
  if (std::all_of(h->tip_table_valid.begin(), h->tip_table_valid.end(), [](char v) { return v != 0; }))
    return PLK_OK;
  if (!h->table_set) return fail(h, PLK_ERR_STATE, "code table not set (plk_set_code_table)");
  for (int t = 0; t < h->n_tips; ++t)
    if (!h->pmat_valid[t]) return fail(h, PLK_ERR_STATE, "transition matrix of tip branch %d not set", t);
  if (h->n_tips > 0) {
    dim3 grid(h->n_tips, h->C);
    if (h->S == 64)
      tip_table64_kernel<<<grid, 256, (size_t)(64 * 64 + h->n_codes * 64) * sizeof(double), h->stream>>>(
          h->pmats, h->code_table, h->tipP, h->n_tips, h->C, h->n_codes);
    else
      tip_table_kernel<<<grid, 256, 0, h->stream>>>(h->pmats, h->code_table, h->tipP, h->n_tips, h->C, h->S,
                                                    h->n_codes);
    HIPCHK(h, hipGetLastError());
  }
  std::fill(h->tip_table_valid.begin(), h->tip_table_valid.end(), 1);
  return PLK_OK;
}

// Device code table in the compact numbering (rows of the codes in use; at least one
// row so that every kernel sees a valid table before the first tip upload).
int upload_compact_table(plk_handle h) {
  const int S = h->S;
  const int U = std::max((int)h->code_orig.size(), 1);
  std::vector<double> t((size_t)U * S, 0.0);
  for (size_t k = 0; k < h->code_orig.size(); ++k)
    std::copy(h->code_table_host.begin() + (size_t)h->code_orig[k] * S,
              h->code_table_host.begin() + (size_t)(h->code_orig[k] + 1) * S, t.begin() + k * S);
  hipSetDevice(h->device);
  HIPCHK(h, hipStreamSynchronize(h->stream));
  HIPCHK(h, hipMemcpy(h->code_table, t.data(), t.size() * sizeof(double), hipMemcpyHostToDevice));
  h->n_codes = U;
  h->tip_table_valid.assign(h->n_tips, 0);
  return PLK_OK;
}

// ---------------------------------------------------------------------------
// Multi-device handle (plk_create_multi): the parent forwards every call to its shards.
// ---------------------------------------------------------------------------
int multi_forward(plk_handle h, int rc) {
  if (rc) {
    h->last_error = std::string("shard: ") + g_last_error;
    for (plk_handle s : h->shards)
      if (!s->last_error.empty()) h->last_error = "shard: " + s->last_error;
  }
  return rc;
}

// f(i) for every shard i, on the shards' host workers (ShardPool); the first failing shard in
// shard order is reported
int multi_run(plk_handle h, const std::function<int(size_t)>& f) {
  const size_t n = h->shards.size();
  if (n == 1) {
    const int rc = f(0);
    if (rc) return fail(h, rc, "shard 0 (device %d): %s", h->shards[0]->device, h->shards[0]->last_error.c_str());
    return PLK_OK;
  }
  if (!h->pool) h->pool.reset(new ShardPool(n));
  h->pool->run(f);
  for (size_t i = 0; i < n; ++i)
    if (const int rc = h->pool->rc[i])
      return fail(h, rc, "shard %zu (device %d): %s", i, h->shards[i]->device, h->shards[i]->last_error.c_str());
  return PLK_OK;
}

int multi_each(plk_handle h, const std::function<int(plk_handle)>& f) {
  return multi_run(h, [&](size_t i) { return f(h->shards[i]); });
}

// f(shard, first pattern of the shard): per-pattern arrays are sliced at the shard starts
int multi_slices(plk_handle h, const std::function<int(plk_handle, int64_t)>& f) {
  return multi_run(h, [&](size_t i) { return f(h->shards[i], h->shard_start[i]); });
}

}  // namespace

extern "C" {
int root_launch_c(plk_handle h, int root, double* site_lnl);
int root_finish_c(plk_handle h, double* lnl, double* block_sums);
}

namespace {
double* block_target(plk_handle h);
void launch_cls_blocks(plk_handle h, int guard, int32_t* uflow, bool site);

// The root reductions of an unscaled handle flag a site likelihood below 2^-255 (or <= 0, or
// NaN) in mapped host memory (plk_root_underflow); a scaled handle's reductions see rescaled
// values, so they get no flag.  The host clears it before a launch that reduces the root.
int32_t* uflow_arm(plk_handle h) {
  if (h->flags & PLK_FLAG_SCALING) return nullptr;
  *(volatile int32_t*)h->h_uflow = 0;
  return h->d_uflow;
}

// first block sum of each shard in the handle's global block order
size_t shard_block0(plk_handle h, size_t i) { return (size_t)(h->shard_start[i] / kRootBlock); }

// the lnL is the sum of all block sums in global block order (bitwise the single-device value)
void sum_blocks(const std::vector<double>& all, double* lnl, double* block_sums) {
  double s = 0.0;
  for (double v : all) s += v;
  if (lnl) *lnl = s;
  if (block_sums) std::memcpy(block_sums, all.data(), all.size() * sizeof(double));
}

int multi_root_loglik_impl(plk_handle h, int root, double* lnl, double* site_lnl, double* block_sums) {
  std::vector<double> all((size_t)h->n_blocks);
  const int rc = multi_run(h, [&](size_t i) {
    plk_handle x = h->shards[i];
    const int r = root_launch_c(x, root, site_lnl ? site_lnl + h->shard_start[i] : nullptr);
    return r ? r : root_finish_c(x, nullptr, all.data() + shard_block0(h, i));
  });
  if (rc) return rc;
  sum_blocks(all, lnl, block_sums);
  return PLK_OK;
}

// every shard's whole evaluation (P(t), traversal, block sums, its stream wait) on its own host
// worker; the fan-out timestamps of plk_get_fanout are taken here
int multi_evaluate(plk_handle h, int n, const int32_t* branch, const int32_t* model, const double* t,
                   const plk_op* ops, int n_ops, int root, double* lnl, double* block_sums) {
  std::vector<double> all((size_t)h->n_blocks);
  const int rc = multi_run(h, [&](size_t i) {
    return plk_evaluate(h->shards[i], n, branch, model, t, ops, n_ops, root, nullptr, all.data() + shard_block0(h, i));
  });
  if (rc) return rc;
  sum_blocks(all, lnl, block_sums);
  const size_t ns = h->shards.size();
  if (ns > 1) {
    const ShardPool& p = *h->pool;
    auto us = [&](clk::time_point b) { return std::chrono::duration<double, std::micro>(b - p.t_post).count(); };
    h->fan_us.resize(3 * ns, 0.0);
    double lo = 1e300, hi = -1e300;
    for (size_t i = 0; i < ns; ++i) {
      const double l = us(h->shards[i]->t_launched);
      h->fan_us[3 * i] += us(p.t_start[i]);
      h->fan_us[3 * i + 1] += l;
      h->fan_us[3 * i + 2] += us(h->shards[i]->t_waited);
      lo = std::min(lo, l);
      hi = std::max(hi, l);
    }
    h->fan_spread_sum += hi - lo;
    h->fan_spread_max = std::max(h->fan_spread_max, hi - lo);
    h->fan_n++;
  }
  return PLK_OK;
}

// per-shard values summed in shard order (the order of the former one-thread loop)
int multi_branch_derivatives(plk_handle h, int branch, double* d1, double* d2) {
  std::vector<double> a(h->shards.size()), b(h->shards.size());
  const int rc = multi_run(h, [&](size_t i) { return plk_branch_derivatives(h->shards[i], branch, &a[i], &b[i]); });
  if (rc) return rc;
  double s1 = 0.0, s2 = 0.0;
  for (size_t i = 0; i < a.size(); ++i) {
    s1 += a[i];
    s2 += b[i];
  }
  if (d1) *d1 = s1;
  if (d2) *d2 = s2;
  return PLK_OK;
}

int multi_all_branch_derivatives(plk_handle h, double* d1, double* d2) {
  const size_t n = (size_t)h->n_nodes, ns = h->shards.size();
  std::vector<double> a(n * ns), b(n * ns), s1(n, 0.0), s2(n, 0.0);
  const int rc = multi_run(h, [&](size_t k) { return plk_all_branch_derivatives(h->shards[k], &a[k * n], &b[k * n]); });
  if (rc) return rc;
  for (size_t k = 0; k < ns; ++k)
    for (size_t i = 0; i < n; ++i) {
      s1[i] += a[k * n + i];
      s2[i] += b[k * n + i];
    }
  if (d1) std::memcpy(d1, s1.data(), n * sizeof(double));
  if (d2) std::memcpy(d2, s2.data(), n * sizeof(double));
  return PLK_OK;
}

int multi_compressed_work(plk_handle h, int64_t* updates) {
  int64_t s = 0;
  for (size_t i = 0; i < h->shards.size(); ++i) {
    int64_t u = 0;
    if (const int r = plk_compressed_work(h->shards[i], &u)) return fail(h, r, "shard %zu: %s", i, h->shards[i]->last_error.c_str());
    s += u;
  }
  if (updates) *updates = s;
  return PLK_OK;
}

int multi_traversal_work(plk_handle h, plk_work* out) {
  plk_work sum;
  std::memset(&sum, 0, sizeof(sum));
  sum.exact = 1;
  for (size_t i = 0; i < h->shards.size(); ++i) {
    plk_work w;
    if (const int r = plk_traversal_work(h->shards[i], &w)) return fail(h, r, "shard %zu: %s", i, h->shards[i]->last_error.c_str());
    sum.patterns += w.patterns;
    sum.node_updates += w.node_updates;
    sum.table_nodes = w.table_nodes;
    sum.table_rows += w.table_rows;
    sum.useful_flops += w.useful_flops;
    sum.issued_flops += w.issued_flops;
    sum.table_flops += w.table_flops;
    sum.exact = sum.exact && w.exact;
    sum.internal_nodes = w.internal_nodes;
  }
  if (out) *out = sum;
  return PLK_OK;
}

}  // namespace

extern "C" {

int plk_abi_version(void) { return PLK_ABI_VERSION; }

#ifndef PLK_SOURCE_HASH
#define PLK_SOURCE_HASH "unknown"
#endif
const char* plk_build_id(void) { return PLK_SOURCE_HASH; }

int plk_block_size(void) { return kRootBlock; }

int plk_device_count(int* count) {
  if (!count) return fail(nullptr, PLK_ERR_ARG, "null count");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    *count = 0;
    return fail(nullptr, PLK_ERR_DEVICE, "hipGetDeviceCount: %s", hipGetErrorString(e));
  }
  *count = n;
  return PLK_OK;
}

const char* plk_last_error(plk_handle h) { return h ? h->last_error.c_str() : g_last_error.c_str(); }

int plk_create(int device, int n_states, int n_classes, int64_t n_patterns, int n_tips, int n_internal,
               int n_models, unsigned flags, plk_handle* out) {
  env_refresh();
  if (!out) return fail(nullptr, PLK_ERR_ARG, "null out handle");
  *out = nullptr;
  if (n_states < 2 || n_states > 64) return fail(nullptr, PLK_ERR_UNSUPPORTED, "n_states %d not in [2, 64]", n_states);
  if (n_classes < 1 || n_classes > 16) return fail(nullptr, PLK_ERR_UNSUPPORTED, "n_classes %d not in [1, 16]", n_classes);
  if ((flags & PLK_FLAG_SUBTREE_PATTERNS) && (flags & PLK_FLAG_DOUBLE_RECURSIVE))
    return fail(nullptr, PLK_ERR_UNSUPPORTED, "double-recursive derivatives read full-length partials (no pattern compression)");
  if (n_patterns < 1 || n_tips < 0 || n_internal < 1 || n_models < 1)
    return fail(nullptr, PLK_ERR_ARG, "bad sizes (patterns %lld tips %d internal %d models %d)",
                (long long)n_patterns, n_tips, n_internal, n_models);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail(nullptr, PLK_ERR_DEVICE, "no HIP device available (libplk has no CPU fallback)");
  if (device < 0 || device >= ndev) return fail(nullptr, PLK_ERR_DEVICE, "device %d out of range (%d devices)", device, ndev);
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess)
    return fail(nullptr, PLK_ERR_DEVICE, "hipGetDeviceProperties failed");
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(nullptr, PLK_ERR_DEVICE, "device %d is %s; libplk is built for gfx950 only", device, prop.gcnArchName);
  if (hipSetDevice(device) != hipSuccess) return fail(nullptr, PLK_ERR_DEVICE, "hipSetDevice(%d) failed", device);

  plk_handle h = new plk_handle_s();
  h->device = device;
  h->S = n_states;
  h->C = n_classes;
  h->n_tips = n_tips;
  h->n_internal = n_internal;
  h->n_nodes = n_tips + n_internal;
  h->n_models = n_models;
  h->flags = flags;
  h->n_patterns = n_patterns;
  h->n_tiles = (int)(((n_patterns + 255) / 256) * 2);  // n_pad multiple of 256 (fused kernel blocks)
  h->n_pad = (int64_t)h->n_tiles * kTile;
  h->n_blocks = (int)((n_patterns + kRootBlock - 1) / kRootBlock);
  h->slot_stride = (int64_t)h->n_tiles * n_classes * n_states * kTile;
  const bool dr = (flags & PLK_FLAG_DOUBLE_RECURSIVE) != 0;
  h->n_mats = h->n_nodes + kScratchMats + (dr ? h->n_nodes : 0);
  h->dr_slot0 = n_internal + kDerivScratch;
  const int n_slots = n_internal + kDerivScratch + (dr ? h->n_nodes : 0);
  h->topo_kids.assign(h->n_nodes, std::vector<int>());
  h->pmat_valid.assign(h->n_nodes, 0);
  h->eigen_set.assign(n_models, 0);
  h->tip_set.assign(n_tips, 0);
  h->tip_table_valid.assign(n_tips, 0);
  int rc = PLK_OK;
  auto bail = [&](int code) {
    plk_destroy(h);
    return code;
  };
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess)
    return bail(fail(nullptr, PLK_ERR_DEVICE, "hipStreamCreate failed"));
  const size_t S2 = (size_t)n_states * n_states;
  // kDerivScratch extra slots / scale rows, kScratchTips extra tip rows and kScratchMats
  // extra transition matrices: scratch for the path derivatives of plk_branch_derivatives (S != 4 path) and
  // plk_root_pair_derivatives;
  // with PLK_FLAG_DOUBLE_RECURSIVE one more slot and matrix per node (U_v, M_f)
  if ((rc = dalloc(h, (void**)&h->partials, (size_t)n_slots * h->slot_stride * sizeof(double)))) return bail(rc);
  if (flags & PLK_FLAG_SCALING) {
    if ((rc = dalloc(h, (void**)&h->scale, (size_t)n_slots * h->n_pad * sizeof(int32_t)))) return bail(rc);
  }
  if ((rc = dalloc(h, (void**)&h->codes, (size_t)(n_tips + kScratchTips) * h->n_pad))) return bail(rc);
  if ((rc = dalloc(h, (void**)&h->pmats, (size_t)h->n_mats * n_classes * S2 * sizeof(double)))) return bail(rc);
  if ((rc = dalloc(h, (void**)&h->V, (size_t)n_models * S2 * sizeof(double)))) return bail(rc);
  if ((rc = dalloc(h, (void**)&h->Vinv, (size_t)n_models * S2 * sizeof(double)))) return bail(rc);
  if ((rc = dalloc(h, (void**)&h->lambda, (size_t)n_models * n_states * sizeof(double)))) return bail(rc);
  if ((rc = dalloc(h, (void**)&h->weights, (size_t)h->n_pad * sizeof(double)))) return bail(rc);
  if ((rc = dalloc(h, (void**)&h->rates, 16 * sizeof(double)))) return bail(rc);
  if ((rc = dalloc(h, (void**)&h->probs, 16 * sizeof(double)))) return bail(rc);
  if ((rc = dalloc(h, (void**)&h->pi, 64 * sizeof(double)))) return bail(rc);
  if ((rc = dalloc(h, (void**)&h->site_lnl, (size_t)h->n_pad * sizeof(double)))) return bail(rc);
  // block sums go straight to pinned host memory (the kernel writes them through the
  // mapped device address), so the evaluation needs no separate device-to-host copy
  if (hipHostMalloc((void**)&h->h_blocks, (size_t)h->n_blocks * sizeof(double), hipHostMallocMapped) != hipSuccess ||
      hipHostGetDevicePointer((void**)&h->block_sums, h->h_blocks, 0) != hipSuccess)
    return bail(fail(h, PLK_ERR_OOM, "pinned block-sum buffer"));
  if ((rc = dalloc(h, (void**)&h->wave_sums, (size_t)(h->n_pad / 64) * sizeof(double)))) return bail(rc);
  if (hipHostMalloc((void**)&h->h_uflow, 64, hipHostMallocMapped) != hipSuccess ||
      hipHostGetDevicePointer((void**)&h->d_uflow, h->h_uflow, 0) != hipSuccess)
    return bail(fail(h, PLK_ERR_OOM, "pinned underflow flag"));
  *h->h_uflow = 0;
  h->materialized.assign(n_internal, 0);
  // default weights 1 for real patterns, 0 for padding
  std::vector<double> w(h->n_pad, 0.0);
  std::fill(w.begin(), w.begin() + n_patterns, 1.0);
  if (hipMemcpy(h->weights, w.data(), w.size() * sizeof(double), hipMemcpyHostToDevice) != hipSuccess)
    return bail(fail(nullptr, PLK_ERR_DEVICE, "weights upload failed"));
  if (hipMemset(h->codes, 0, (size_t)std::max(n_tips, 1) * h->n_pad) != hipSuccess)
    return bail(fail(nullptr, PLK_ERR_DEVICE, "codes memset failed"));
  if (h->scale && hipMemset(h->scale, 0, (size_t)n_internal * h->n_pad * sizeof(int32_t)) != hipSuccess)
    return bail(fail(nullptr, PLK_ERR_DEVICE, "scale memset failed"));
  *out = h;
  return PLK_OK;
}

void comm_release(plk_handle h);

int plk_destroy(plk_handle h) {
  if (!h) return PLK_OK;
  if (!h->shards.empty()) {
    h->pool.reset();  // workers joined before their shards go
    for (plk_handle s : h->shards) plk_destroy(s);
    delete h;
    return PLK_OK;
  }
  hipSetDevice(h->device);
  if (h->stream) hipStreamSynchronize(h->stream);
  comm_release(h);
  void* bufs[] = {h->partials, h->scale, h->codes, h->code_table, h->tipP, h->pmats, h->dpmats, h->d2pmats,
                  h->V, h->Vinv, h->lambda, h->weights, h->rates, h->probs, h->pi, h->site_lnl,
                  h->d_ops, h->wave_sums, h->d_links, h->d_opsl, h->d_prog, h->d_frag, h->d1_sums,
                  h->d2_sums, h->d_dprog, h->pmatsT, h->d_ucodes, h->d_units, h->d_cherry3,
                  h->d_cherry_tips, h->d_cherry, h->d_drb, h->d_drm, h->dr_blk, h->dr_out, h->d_drpre, h->d_sbctr,
                  h->d_cherry_rows, h->d_kidsl, h->d_cls, h->d_ucodes_dc, h->d_units_start};
  for (void* p : bufs)
    if (p) hipFree(p);
  if (h->h_req) (void)hipHostFree(h->h_req);
  if (h->h_blocks) hipHostFree(h->h_blocks);
  if (h->h_uflow) hipHostFree(h->h_uflow);
  if (h->h_clk) hipHostFree(h->h_clk);
  if (h->req_done) hipEventDestroy(h->req_done);
  for (auto& e : h->events) {
    hipEventDestroy(e.a);
    hipEventDestroy(e.b);
  }
  for (auto& e : h->event_pool) {
    hipEventDestroy(e.a);
    hipEventDestroy(e.b);
  }
  if (h->stream) hipStreamDestroy(h->stream);
  delete h;
  return PLK_OK;
}

int plk_comm_get_id(plk_comm_id* id) {
  env_refresh();
  if (!id) return fail(nullptr, PLK_ERR_ARG, "null id");
  static_assert(sizeof(plk_comm_id) == sizeof(ncclUniqueId), "plk_comm_id wraps ncclUniqueId");
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return fail(nullptr, PLK_ERR_DEVICE, "ncclGetUniqueId failed");
  std::memcpy(id->internal, u.internal, sizeof(u.internal));
  return PLK_OK;
}

// Tear down a communicator and its exchange buffers (a failed plk_comm_init leaves the
// handle on the single-rank path, as before the call).
void comm_release(plk_handle h) {
  if (h->comm) ncclCommDestroy(h->comm);
  h->comm = nullptr;
  for (void* p : {(void*)h->d_blk_local, (void*)h->d_blk_all, (void*)h->d_comm_counts, (void*)h->d_xch,
                  (void*)h->d_xch_all})
    if (p) hipFree(p);
  h->d_blk_local = h->d_blk_all = h->d_xch = h->d_xch_all = nullptr;
  h->d_xch_cap = h->d_xch_all_cap = 0;
  h->d_comm_counts = nullptr;
  if (h->h_blk_all) hipHostFree(h->h_blk_all);
  h->h_blk_all = nullptr;
  h->d_blk_all_map = nullptr;
  h->comm_counts.clear();
  h->comm_ranks = 0;
  h->comm_rank = 0;
  h->comm_stride = 0;
  h->comm_uflow = 0;
}

int plk_comm_init(plk_handle h, int n_ranks, int rank, const plk_comm_id* id) {
  env_refresh();
  if (!h || !id || n_ranks < 1 || rank < 0 || rank >= n_ranks) return fail(h, PLK_ERR_ARG, "bad communicator arguments");
  if (!h->shards.empty()) return fail(h, PLK_ERR_UNSUPPORTED, "a multi-device handle exchanges in-process");
  if (h->comm) return fail(h, PLK_ERR_STATE, "communicator already initialised");
  hipSetDevice(h->device);
  ncclUniqueId u;
  std::memcpy(u.internal, id->internal, sizeof(u.internal));
  if (ncclCommInitRank(&h->comm, n_ranks, u, rank) != ncclSuccess) {
    h->comm = nullptr;
    return fail(h, PLK_ERR_DEVICE, "ncclCommInitRank(%d ranks, rank %d) failed", n_ranks, rank);
  }
  int64_t* d_one = nullptr;
  // every failure after the communicator exists goes through comm_release
  auto setup = [&]() -> int {
    // block counts of every rank, once: per evaluation the all-gather has a fixed size
    int rc = dalloc(h, (void**)&h->d_comm_counts, (size_t)n_ranks * sizeof(int64_t));
    if (rc) return rc;
    if ((rc = dalloc(h, (void**)&d_one, sizeof(int64_t)))) return rc;
    const int64_t mine = h->n_blocks;
    HIPCHK(h, hipMemcpy(d_one, &mine, sizeof(int64_t), hipMemcpyHostToDevice));
    if (ncclAllGather(d_one, h->d_comm_counts, 1, ncclInt64, h->comm, h->stream) != ncclSuccess)
      return fail(h, PLK_ERR_DEVICE, "ncclAllGather of the block counts failed");
    std::vector<int64_t> counts((size_t)n_ranks);
    HIPCHK(h, hipMemcpyAsync(counts.data(), h->d_comm_counts, counts.size() * sizeof(int64_t),
                             hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    // PLK_TEST_COMM_PAD=k (test hook): k more padding doubles per record, so that a one-rank
    // run exercises the zero padding a rank with fewer blocks than another carries
    const char* pad = env_get("PLK_TEST_COMM_PAD");
    const int64_t stride = xchg::stride(counts.data(), n_ranks) + (pad ? std::max(0, std::atoi(pad)) : 0);
    if (stride < 1) return fail(h, PLK_ERR_ARG, "bad block counts in the exchange");
    if ((rc = dalloc(h, (void**)&h->d_blk_local, (size_t)stride * sizeof(double)))) return rc;
    if ((rc = dalloc(h, (void**)&h->d_blk_all, (size_t)n_ranks * stride * sizeof(double)))) return rc;
    HIPCHK(h, hipMemset(h->d_blk_local, 0, (size_t)stride * sizeof(double)));
    if (hipHostMalloc((void**)&h->h_blk_all, (size_t)n_ranks * stride * sizeof(double), hipHostMallocMapped) !=
            hipSuccess ||
        hipHostGetDevicePointer((void**)&h->d_blk_all_map, h->h_blk_all, 0) != hipSuccess)
      return fail(h, PLK_ERR_OOM, "pinned block sums of every rank");
    h->comm_stride = stride;
    h->comm_counts = counts;
    return PLK_OK;
  };
  int rc = env_is("PLK_TEST_COMM_FAIL", '1') ? fail(h, PLK_ERR_OOM, "forced exchange-setup failure (test)") : setup();
  if (d_one) hipFree(d_one);
  if (rc) {
    comm_release(h);
    return rc;
  }
  h->comm_ranks = n_ranks;
  h->comm_rank = rank;
  return PLK_OK;
}

int plk_set_code_table(plk_handle h, int n_codes, const double* code_to_vec) {
  env_refresh();
  if (h && !h->shards.empty()) return multi_each(h, [&](plk_handle x) { return plk_set_code_table(x, n_codes, code_to_vec); });
  if (!h || !code_to_vec || n_codes < 1 || n_codes > 256) return fail(h, PLK_ERR_ARG, "bad code table (n_codes %d)", n_codes);
  if (h->S == 4 && n_codes > kMaxCodes4 && s4_supported(h->C))
    return fail(h, PLK_ERR_UNSUPPORTED, "4-state engine supports at most %d codes", kMaxCodes4);
  for (int c : h->code_orig)
    if (c >= n_codes)
      return fail(h, PLK_ERR_STATE, "uploaded tip codes use code %d, outside the new table (%d codes)", c, n_codes);
  hipSetDevice(h->device);
  HIPCHK(h, hipStreamSynchronize(h->stream));
  if (h->code_table) hipFree(h->code_table);
  if (h->tipP) hipFree(h->tipP);
  h->code_table = nullptr;
  h->tipP = nullptr;
  int rc;
  if ((rc = dalloc(h, (void**)&h->code_table, (size_t)n_codes * h->S * sizeof(double)))) return rc;
  if ((rc = dalloc(h, (void**)&h->tipP, (size_t)(h->n_tips + kScratchTips) * h->C * n_codes * h->S * sizeof(double))))
    return rc;
  h->code_table_host.assign(code_to_vec, code_to_vec + (size_t)n_codes * h->S);
  h->n_codes_table = n_codes;
  h->code_map.resize(256, -1);
  h->table_set = true;
  return upload_compact_table(h);
}

int plk_set_tip_codes(plk_handle h, int tip, const uint8_t* codes) {
  env_refresh();
  if (h && !h->shards.empty()) return multi_slices(h, [&](plk_handle x, int64_t a) { return plk_set_tip_codes(x, tip, codes ? codes + a : nullptr); });
  if (!h || !codes || tip < 0 || tip >= h->n_tips) return fail(h, PLK_ERR_ARG, "bad tip index %d", tip);
  if (!h->table_set) return fail(h, PLK_ERR_STATE, "plk_set_code_table must precede plk_set_tip_codes");
  bool seen[256] = {false};
  for (int64_t i = 0; i < h->n_patterns; ++i) seen[codes[i]] = true;
  for (int c = 0; c < 256; ++c)
    if (seen[c] && c >= h->n_codes_table) {
      int64_t i = 0;
      while (codes[i] != c) ++i;
      return fail(h, PLK_ERR_BAD_CODE, "tip %d pattern %lld: code %d outside the code table (%d codes)", tip,
                  (long long)i, c, h->n_codes_table);
    }
  bool grown = false;
  for (int c = 0; c < 256; ++c)
    if (seen[c] && h->code_map[c] < 0) {
      h->code_map[c] = (int)h->code_orig.size();
      h->code_orig.push_back(c);
      grown = true;
    }
  if (grown) {
    int rc = upload_compact_table(h);
    if (rc) return rc;
  }
  std::vector<uint8_t> cc((size_t)h->n_patterns);
  for (int64_t i = 0; i < h->n_patterns; ++i) cc[(size_t)i] = (uint8_t)h->code_map[codes[i]];
  if (h->flags & PLK_FLAG_SUBTREE_PATTERNS) {
    if (h->tip_codes_host.empty()) h->tip_codes_host.resize(h->n_tips);
    h->tip_codes_host[tip] = cc;
    h->cmp_valid = false;
  }
  hipSetDevice(h->device);
  HIPCHK(h, hipMemcpy(h->codes + (size_t)tip * h->n_pad, cc.data(), (size_t)h->n_patterns, hipMemcpyHostToDevice));
  h->tip_set[tip] = 1;
  h->ucodes_valid = false;
  h->cherry_codes_valid = false;
  return PLK_OK;
}

int plk_set_pattern_weights(plk_handle h, const double* weights) {
  env_refresh();
  if (h && !h->shards.empty()) return multi_slices(h, [&](plk_handle x, int64_t a) { return plk_set_pattern_weights(x, weights ? weights + a : nullptr); });
  if (!h || !weights) return fail(h, PLK_ERR_ARG, "null weights");
  hipSetDevice(h->device);
  HIPCHK(h, hipStreamSynchronize(h->stream));
  HIPCHK(h, hipMemcpy(h->weights, weights, (size_t)h->n_patterns * sizeof(double), hipMemcpyHostToDevice));
  h->fused_lnl_valid = false;  // a cached fused root reduction used the old weights
  return PLK_OK;
}

int plk_set_category_rates(plk_handle h, const double* rates, const double* probs) {
  env_refresh();
  if (h && !h->shards.empty()) return multi_each(h, [&](plk_handle x) { return plk_set_category_rates(x, rates, probs); });
  if (!h || !rates || !probs) return fail(h, PLK_ERR_ARG, "null rates/probs");
  hipSetDevice(h->device);
  HIPCHK(h, hipStreamSynchronize(h->stream));
  HIPCHK(h, hipMemcpy(h->rates, rates, h->C * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(h, hipMemcpy(h->probs, probs, h->C * sizeof(double), hipMemcpyHostToDevice));
  h->rates_set = true;
  h->fused_lnl_valid = false;  // a cached fused root reduction used the old class probabilities
  return PLK_OK;
}

int plk_set_root_frequencies(plk_handle h, const double* pi) {
  env_refresh();
  if (h && !h->shards.empty()) return multi_each(h, [&](plk_handle x) { return plk_set_root_frequencies(x, pi); });
  if (!h || !pi) return fail(h, PLK_ERR_ARG, "null frequencies");
  hipSetDevice(h->device);
  HIPCHK(h, hipStreamSynchronize(h->stream));
  HIPCHK(h, hipMemcpy(h->pi, pi, h->S * sizeof(double), hipMemcpyHostToDevice));
  h->pi_set = true;
  h->fused_lnl_valid = false;  // a cached fused root reduction used the old frequencies
  return PLK_OK;
}

int plk_set_eigen(plk_handle h, int model, const double* V, const double* Vinv, const double* lambda) {
  env_refresh();
  if (h && !h->shards.empty()) return multi_each(h, [&](plk_handle x) { return plk_set_eigen(x, model, V, Vinv, lambda); });
  if (!h || !V || !Vinv || !lambda || model < 0 || model >= h->n_models)
    return fail(h, PLK_ERR_ARG, "bad eigen system (model %d)", model);
  hipSetDevice(h->device);
  HIPCHK(h, hipStreamSynchronize(h->stream));
  const size_t S2 = (size_t)h->S * h->S;
  HIPCHK(h, hipMemcpy(h->V + model * S2, V, S2 * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(h, hipMemcpy(h->Vinv + model * S2, Vinv, S2 * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(h, hipMemcpy(h->lambda + (size_t)model * h->S, lambda, h->S * sizeof(double), hipMemcpyHostToDevice));
  h->eigen_set[model] = 1;
  return PLK_OK;
}

int plk_update_pmatrices(plk_handle h, int n, const int32_t* branch, const int32_t* model, const double* t,
                         unsigned deriv_mask) {
  env_refresh();
  if (h && !h->shards.empty()) return multi_each(h, [&](plk_handle x) { return plk_update_pmatrices(x, n, branch, model, t, deriv_mask); });
  if (!h || n < 0 || (n > 0 && (!branch || !t))) return fail(h, PLK_ERR_ARG, "bad pmatrix request");
  if (n == 0) return PLK_OK;
  if (!h->rates_set) return fail(h, PLK_ERR_STATE, "plk_set_category_rates must precede plk_update_pmatrices");
  if (deriv_mask == 0) deriv_mask = PLK_DERIV_P;
  for (int i = 0; i < n; ++i) {
    if (branch[i] < 0 || branch[i] >= h->n_nodes) return fail(h, PLK_ERR_ARG, "branch %d out of range", branch[i]);
    const int m = model ? model[i] : 0;
    if (m < 0 || m >= h->n_models) return fail(h, PLK_ERR_ARG, "model %d out of range", m);
    if (!h->eigen_set[m]) return fail(h, PLK_ERR_STATE, "eigen system %d not set", m);
    if (!(t[i] >= 0.0)) return fail(h, PLK_ERR_ARG, "branch length %g not >= 0", t[i]);
  }
  hipSetDevice(h->device);
  const size_t S2 = (size_t)h->S * h->S;
  if ((deriv_mask & PLK_DERIV_DP) && !h->dpmats) {
    int rc = dalloc(h, (void**)&h->dpmats, (size_t)h->n_nodes * h->C * S2 * sizeof(double));
    if (rc) return rc;
  }
  if ((deriv_mask & PLK_DERIV_D2P) && !h->d2pmats) {
    int rc = dalloc(h, (void**)&h->d2pmats, (size_t)h->n_nodes * h->C * S2 * sizeof(double));
    if (rc) return rc;
  }
  // small requests ride in the kernel arguments; larger ones go through pinned staging
  // and a stream-ordered copy (the host only waits for the previous request's copy)
  static_assert(sizeof(PmatInline) + sizeof(PmatArgs) <= 4096, "kernel argument block");
  PmatInline inl;
  inl.n = 0;
  const size_t off_t = 0, off_b = (size_t)n * sizeof(double), off_m = off_b + (size_t)n * sizeof(int32_t);
  if (n <= kPmatInline) {
    inl.n = n;
    for (int i = 0; i < n; ++i) {
      inl.t[i] = t[i];
      inl.branch[i] = branch[i];
      inl.model[i] = model ? model[i] : 0;
    }
  }
  // larger requests: a staging buffer the host writes and the kernel reads (cfg5, 1 022
  // branches: 8.6 us less per evaluation than a stream-ordered copy into device memory -- the
  // copy's launch and host API time); see req_staging for where it lives.  The host rewrites
  // the staging only after the previous request's reader finished (req_done, or the stream
  // wait that ends plk_evaluate).
  const char* req = nullptr;
  if (inl.n == 0) {
    const size_t bytes = (size_t)n * (2 * sizeof(int32_t) + sizeof(double)) + 64;
    if (!h->req_done) HIPCHK(h, hipEventCreateWithFlags(&h->req_done, hipEventDisableTiming));
    if (h->req_unrecorded) {
      HIPCHK(h, hipStreamSynchronize(h->stream));
      h->req_unrecorded = false;
    } else {
      HIPCHK(h, hipEventSynchronize(h->req_done));
    }
    int rc = req_staging(h, bytes);
    if (rc) return rc;
    char* staging = h->h_req;
    std::memcpy(staging + off_t, t, n * sizeof(double));
    // an optimiser's evaluations repeat the branch and model arrays: those stores (over the
    // BAR for a device-memory staging) are skipped when the staging already holds them
    // (shadow: n, model given, then the arrays as written)
    const size_t nb = 2 + (size_t)n * (model ? 2 : 1);
    const bool same = h->req_shadow.size() == nb && h->req_shadow[0] == n && h->req_shadow[1] == (model ? 1 : 0) &&
                      std::memcmp(h->req_shadow.data() + 2, branch, n * sizeof(int32_t)) == 0 &&
                      (!model || std::memcmp(h->req_shadow.data() + 2 + n, model, n * sizeof(int32_t)) == 0);
    if (!same) {
      std::memcpy(staging + off_b, branch, n * sizeof(int32_t));
      if (model) std::memcpy(staging + off_m, model, n * sizeof(int32_t));
      h->req_shadow.assign({n, model ? 1 : 0});
      h->req_shadow.insert(h->req_shadow.end(), branch, branch + n);
      if (model) h->req_shadow.insert(h->req_shadow.end(), model, model + n);
    }
    // the host's stores reach the staging before the launch's doorbell (a device-memory
    // staging is write-combined over the BAR)
    std::atomic_thread_fence(std::memory_order_seq_cst);
    req = h->h_req_dev;
  }
  PmatArgs a;
  a.t = inl.n ? nullptr : reinterpret_cast<const double*>(req + off_t);
  a.branch = inl.n ? nullptr : reinterpret_cast<const int32_t*>(req + off_b);
  a.model = (model && !inl.n) ? reinterpret_cast<const int32_t*>(req + off_m) : nullptr;
  a.rates = h->rates;
  a.V = h->V;
  a.Vinv = h->Vinv;
  a.lambda = h->lambda;
  a.P = h->pmats;
  a.PT = nullptr;
  a.dP = h->dpmats;
  a.d2P = h->d2pmats;
  a.S = h->S;
  a.C = h->C;
  a.mask = deriv_mask;
  a.n_req = n;
  a.uni_model = -1;
  if (h->S == 64) {
    a.uni_model = model ? model[0] : 0;
    for (int i = 1; model && i < n; ++i)
      if (model[i] != a.uni_model) a.uni_model = -1;
  }
  // tip tables ride along for S <= 20 (P of the block staged in LDS; S = 64 keeps the
  // separate tip_table_kernel)
  const bool k64 = h->S == 64 && deriv_mask == PLK_DERIV_P;
  const bool tips_fused = h->table_set && (h->S <= 20 || (k64 && h->n_codes <= 64));
  a.init = tips_fused ? h->code_table : nullptr;
  a.tipP = h->tipP;
  a.n_tips = h->n_tips;
  a.n_codes = h->n_codes;
  EventPair ev;
  if (h->timing & PLK_TIME_PMAT) {
    ev = get_events(h, 1);
    hipEventRecord(ev.a, h->stream);
  }
  const size_t lds = (size_t)(h->S + (tips_fused ? 3 : 2) * S2) * sizeof(double);
  // pmat64s_kernel and pmat_kernel also write the transposed copy the matrix-core kernels
  // read (allocated by the first transposed-P use), so an evaluation needs no transpose launch
  const bool pk_generic = !k64 && h->S != 4;
  if ((k64 || pk_generic) && (deriv_mask & PLK_DERIV_P)) a.PT = h->pmatsT;
  if (k64) {
    // several matrices per workgroup (pmat64w_kernel); PLK_TUNE P64RX=0 keeps pmat64s_kernel
    const int rx = tune_int("P64RX", 4, 0, 4), nb = tune_int("P64NB", 2, 1, 4);
    if (rx == 0) {
      pmat64s_kernel<<<dim3(n, h->C, 4), dim3(256), (size_t)(64 + 16 * 64 + S2) * sizeof(double), h->stream>>>(a, inl);
    } else {
      const int rr = rx <= 1 ? 1 : rx <= 2 ? 2 : 4, nn = nb <= 1 ? 1 : nb <= 2 ? 2 : 4;
      const dim3 g((unsigned)((n * h->C + nn - 1) / nn), (unsigned)(64 / (4 * rr)));
      const size_t lds = (size_t)(64 * kP64Pad + nn * 64 + nn * 4 * rr * kP64Pad) * sizeof(double);
#define PLK_P64W(RX_, NB_) \
  if (rr == RX_ && nn == NB_) pmat64w_kernel<RX_, NB_><<<g, dim3(256), lds, h->stream>>>(a, inl);
      PLK_P64W(1, 1) PLK_P64W(1, 2) PLK_P64W(1, 4) PLK_P64W(2, 1) PLK_P64W(2, 2) PLK_P64W(2, 4)
      PLK_P64W(4, 1) PLK_P64W(4, 2) PLK_P64W(4, 4)
#undef PLK_P64W
    }
  } else if (h->S == 4)
  {
    const dim3 g4((unsigned)((n * h->C * 4 + 63) / 64));
    // <= 64 branches: the 1 KB argument block (cfg2: 0.7 us per evaluation, profiles/r05/ab_runs.md)
    if (inl.n > 0 && inl.n <= kPmatInlineSmall) {
      PmatInlineSmall sm;
      sm.n = inl.n;
      std::copy(inl.t, inl.t + inl.n, sm.t);
      std::copy(inl.branch, inl.branch + inl.n, sm.branch);
      std::copy(inl.model, inl.model + inl.n, sm.model);
      pmat4_kernel<PmatInlineSmall><<<g4, dim3(64), 0, h->stream>>>(a, sm);
    } else {
      pmat4_kernel<PmatInline><<<g4, dim3(64), 0, h->stream>>>(a, inl);
    }
  }
  else
  {
    const int nth = h->S <= 4 ? 64 : 256, ne = (int)((S2 + nth - 1) / nth);
    const dim3 g(n, h->C);
    if (ne <= 1) pmat_kernel<1><<<g, dim3(nth), lds, h->stream>>>(a, inl);
    else if (ne <= 2) pmat_kernel<2><<<g, dim3(nth), lds, h->stream>>>(a, inl);
    else if (ne <= 4) pmat_kernel<4><<<g, dim3(nth), lds, h->stream>>>(a, inl);
    else if (ne <= 8) pmat_kernel<8><<<g, dim3(nth), lds, h->stream>>>(a, inl);
    else pmat_kernel<16><<<g, dim3(nth), lds, h->stream>>>(a, inl);
  }
  HIPCHK(h, hipGetLastError());
  if (inl.n == 0) {
    // the kernel read the staging: plk_evaluate waits for the whole stream before it returns
    // (no record needed), other callers record req_done
    if (h->in_eval)
      h->req_unrecorded = true;
    else
      HIPCHK(h, hipEventRecord(h->req_done, h->stream));
  }
  if (h->timing & PLK_TIME_PMAT) {
    hipEventRecord(ev.b, h->stream);
    h->events.push_back(ev);
  }
  if (deriv_mask & PLK_DERIV_P) {
    for (int i = 0; i < n; ++i) {
      h->pmat_valid[branch[i]] = 1;
      if (!a.PT) h->pmatsT_dirty = true;  // pmat64s_kernel wrote the transposed rows too
      if (branch[i] < h->n_tips) h->tip_table_valid[branch[i]] = tips_fused ? 1 : 0;  // row written by pmat_kernel
    }
  }
  if (h->deriv_valid.empty()) h->deriv_valid.assign(h->n_nodes, 0);
  // dP/d2P stay consistent with P only when all three come from the same call
  const bool both = (deriv_mask & (PLK_DERIV_P | PLK_DERIV_DP | PLK_DERIV_D2P)) ==
                    (PLK_DERIV_P | PLK_DERIV_DP | PLK_DERIV_D2P);
  for (int i = 0; i < n; ++i) h->deriv_valid[branch[i]] = both ? 1 : 0;
  return PLK_OK;
}

int plk_set_pmatrix(plk_handle h, int branch, const double* P) {
  env_refresh();
  if (h && !h->shards.empty()) return multi_each(h, [&](plk_handle x) { return plk_set_pmatrix(x, branch, P); });
  if (!h || !P || branch < 0 || branch >= h->n_nodes) return fail(h, PLK_ERR_ARG, "bad branch %d", branch);
  hipSetDevice(h->device);
  HIPCHK(h, hipStreamSynchronize(h->stream));
  const size_t n = (size_t)h->C * h->S * h->S;
  HIPCHK(h, hipMemcpy(h->pmats + (size_t)branch * n, P, n * sizeof(double), hipMemcpyHostToDevice));
  h->pmat_valid[branch] = 1;
  h->pmatsT_dirty = true;
  if (!h->deriv_valid.empty()) h->deriv_valid[branch] = 0;
  if (branch < h->n_tips) h->tip_table_valid[branch] = 0;
  return PLK_OK;
}

int plk_get_dpmatrix(plk_handle h, int branch, int order, double* dP) {
  env_refresh();
  if (h && !h->shards.empty()) return multi_forward(h, plk_get_dpmatrix(h->shards[0], branch, order, dP));
  if (!h || !dP || branch < 0 || branch >= h->n_nodes || (order != 1 && order != 2))
    return fail(h, PLK_ERR_ARG, "bad derivative request (branch %d, order %d)", branch, order);
  const double* src = order == 1 ? h->dpmats : h->d2pmats;
  if (!src) return fail(h, PLK_ERR_STATE, "no derivative matrices (PLK_DERIV_DP / PLK_DERIV_D2P)");
  hipSetDevice(h->device);
  HIPCHK(h, hipStreamSynchronize(h->stream));
  const size_t n = (size_t)h->C * h->S * h->S;
  HIPCHK(h, hipMemcpy(dP, src + (size_t)branch * n, n * sizeof(double), hipMemcpyDeviceToHost));
  return PLK_OK;
}

int plk_get_pmatrix(plk_handle h, int branch, double* P) {
  env_refresh();
  if (h && !h->shards.empty()) return multi_forward(h, plk_get_pmatrix(h->shards[0], branch, P));
  if (!h || !P || branch < 0 || branch >= h->n_nodes) return fail(h, PLK_ERR_ARG, "bad branch %d", branch);
  hipSetDevice(h->device);
  HIPCHK(h, hipStreamSynchronize(h->stream));
  const size_t n = (size_t)h->C * h->S * h->S;
  HIPCHK(h, hipMemcpy(P, h->pmats + (size_t)branch * n, n * sizeof(double), hipMemcpyDeviceToHost));
  return PLK_OK;
}

}  // extern "C"

namespace {

// ---------------------------------------------------------------------------
// Fused 4-state traversal: program builder + launches (kernel in plk_tree4.hpp).
// ---------------------------------------------------------------------------
// register levels of the interpreter (one wave per rate class: the smallest register
// footprint and the highest occupancy; the generated kernel also puts every class of a
// pattern in one wave, with the same results bitwise)
constexpr int kTree4Levels = 8;

// Fused traversal kernels: 4 states -> the VALU tree kernels (plk_jit.hpp generated per
// tree, tree4_kernel interpreting the same program); 20 states -> jit_treeM (plk_jitm.hpp,
// fp64 MFMA 4x4x4_4b) or the treeM interpreter; 64 states, one class -> treeM (16x16x4).
enum FusedKind { FK_NONE = 0, FK_TREE4, FK_TREEM };

FusedKind fused_kind(plk_handle h) {
  if (h->flags & PLK_FLAG_LEVELWISE) return FK_NONE;
  // 4 states: the VALU tree kernel (plk_jit.hpp); on the 4x4x4 matrix cores (one block per
  // class and 16 patterns) it measured slower
  if (h->S == 4) return (h->C == 1 || h->C == 2 || h->C == 4) ? FK_TREE4 : FK_NONE;
  if (h->C > kTreeMaxWaves) return FK_NONE;
  if (h->S == 20) return FK_TREEM;
  if (h->S == 64 && h->C == 1) return FK_TREEM;  // the treeM interpreter takes one class
  return FK_NONE;
}

bool tree4_supported(plk_handle h) { return fused_kind(h) != FK_NONE; }

int tune_int(const char* key, int def, int lo, int hi) {
  const char* e = tune_get(key);
  if (!e) return def;
  const int v = std::atoi(e);
  return (v >= lo && v <= hi) ? v : def;
}

// 4 states, one class per wave: the tree-specialised kernel (plk_jit.hpp) serves the
// fused traversal; PLK_JIT=0 keeps the interpreter (tree4_kernel), e.g. for A/B runs.
bool jit_tree4(plk_handle h) { return fused_kind(h) == FK_TREE4 && !tune_is("JIT", '0'); }

// 20 states: the tree-specialised kernel on v_mfma_f64_4x4x4_4b (plk_jitm.hpp) serves the
// fused traversal; PLK_JITM=0 keeps the treeM interpreter (16x16x4 MFMA), e.g. for A/B runs.
bool jit_treeM(plk_handle h) {
  if (fused_kind(h) != FK_TREEM || tune_is("JITM", '0')) return false;
  return h->S == 20;
}

// Classes in one wave (plk_jit.hpp, CW = C): the joint rescale needs no cross-wave
// exchange (the per-node barrier of the one-class-per-wave layout costs ~2x on cfg5),
// at the price of C x the registers per level (so a lower fragment height).  Default
// for scaling runs; PLK_JIT_CIW=0/1 overrides.
bool jit_ciw(plk_handle h) {
  if (!jit_tree4(h) || h->C == 1) return false;
  const char* e = tune_get("JIT_CIW");
  if (e) return e[0] == '1';
  return (h->flags & PLK_FLAG_SCALING) != 0;
}

// tips whose tables (C x codes-in-use x 4 doubles each) fit one fragment's LDS budget
int jit_tip_cap(plk_handle h) {
  constexpr int kb = 48;
  return std::max(2, (kb * 1024) / (h->C * std::max(h->n_codes, 1) * 4 * (int)sizeof(double)));
}

// treeM programs replace unstored cherries by T_CHERRY rows; combined codes are 16-bit
bool treeM_cherries(plk_handle h) { return fused_kind(h) == FK_TREEM && h->n_codes * h->n_codes <= 65535; }

// Cherry contribution tables of the current treeM program (plk_treeM.hpp), rebuilt on
// every traversal (P(t) and the tip tables may have changed); combined codes only when
// the tip codes or the program changed.
int build_cherry_tables(plk_handle h) {
  const int nch = (int)h->cherry3.size() / 3;
  if (nch == 0) return PLK_OK;
  const int U = h->n_codes, S = h->S, C = h->C;
  const CherryLayout lay(C, U, S, h->n_pad);
  int rc = ensure_cap(h, (void**)&h->d_cherry, &h->cherry_cap, (size_t)nch * lay.stride);
  if (rc) return rc;
  if (!h->cherry_codes_valid) {
    std::vector<int32_t> tips(2 * (size_t)nch);
    for (int k = 0; k < nch; ++k) {
      tips[2 * (size_t)k] = h->cherry3[3 * (size_t)k];
      tips[2 * (size_t)k + 1] = h->cherry3[3 * (size_t)k + 1];
    }
    rc = ensure_cap(h, (void**)&h->d_cherry3, &h->cherry3_cap, h->cherry3.size() * sizeof(int32_t));
    if (!rc) rc = ensure_cap(h, (void**)&h->d_cherry_tips, &h->cherry_tips_cap, tips.size() * sizeof(int32_t));
    if (rc) return rc;
    HIPCHK(h, hipMemcpyAsync(h->d_cherry3, h->cherry3.data(), h->cherry3.size() * sizeof(int32_t),
                             hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, hipMemcpyAsync(h->d_cherry_tips, tips.data(), tips.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                             h->stream));
    cherry_codes_kernel<<<dim3((unsigned)((h->n_pad + 255) / 256), (unsigned)nch), 256, 0, h->stream>>>(
        h->codes, h->n_pad, h->d_cherry_tips, U, lay, h->d_cherry);
    HIPCHK(h, hipGetLastError());
    // the code pairs each cherry meets: marked on the device, listed here (once per set of
    // tip codes / program)
    const size_t U2 = (size_t)U * U;
    uint8_t* d_mark = nullptr;
    HIPCHK(h, hipMallocAsync((void**)&d_mark, (size_t)nch * U2, h->stream));
    HIPCHK(h, hipMemsetAsync(d_mark, 0, (size_t)nch * U2, h->stream));
    cherry_mark_kernel<<<dim3((unsigned)((h->n_pad + 255) / 256), (unsigned)nch), 256, 0, h->stream>>>(
        h->n_pad, U, lay, h->d_cherry, d_mark);
    HIPCHK(h, hipGetLastError());
    std::vector<uint8_t> mark((size_t)nch * U2);
    HIPCHK(h, hipMemcpyAsync(mark.data(), d_mark, mark.size(), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipFreeAsync(d_mark, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));  // `tips` goes out of scope, `mark` is read
    std::vector<int32_t> rl((size_t)nch + 1, 0);
    h->cherry_rows_max = 0;
    for (int k = 0; k < nch; ++k) {
      for (size_t r = 0; r < U2; ++r)
        if (mark[(size_t)k * U2 + r]) rl.push_back((int32_t)r);
      rl[(size_t)k + 1] = (int32_t)(rl.size() - (size_t)nch - 1);
      h->cherry_rows_max = std::max(h->cherry_rows_max, rl[(size_t)k + 1] - rl[(size_t)k]);
    }
    rc = ensure_cap(h, (void**)&h->d_cherry_rows, &h->cherry_rows_cap, rl.size() * sizeof(int32_t));
    if (rc) return rc;
    HIPCHK(h, hipMemcpy(h->d_cherry_rows, rl.data(), rl.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    h->cherry_codes_valid = true;
  }
  // rows per workgroup (64-row passes sharing one P^T staging): one pass (cfg3 tables
  // 35 us vs 40 at four passes, cfg4 36 vs 38; profiles/r04/ab_runs.md)
  constexpr int rows = 64;
  const dim3 grid((unsigned)((std::max(h->cherry_rows_max, 1) + rows - 1) / rows), (unsigned)(nch * C));
  const int32_t* rs = h->d_cherry_rows;
  const int32_t* rlist = h->d_cherry_rows + nch + 1;
  const bool sc = (h->flags & PLK_FLAG_SCALING) != 0;
  if (S == 20) {
    if (sc) cherry_table_kernel<20, true><<<grid, 256, 0, h->stream>>>(h->tipP, h->pmatsT, h->d_cherry3, C, U, lay, h->d_cherry, rows, rs, rlist);
    else cherry_table_kernel<20, false><<<grid, 256, 0, h->stream>>>(h->tipP, h->pmatsT, h->d_cherry3, C, U, lay, h->d_cherry, rows, rs, rlist);
  } else if (S == 4) {
    if (sc) cherry_table_kernel<4, true><<<grid, 256, 0, h->stream>>>(h->tipP, h->pmatsT, h->d_cherry3, C, U, lay, h->d_cherry, rows, rs, rlist);
    else cherry_table_kernel<4, false><<<grid, 256, 0, h->stream>>>(h->tipP, h->pmatsT, h->d_cherry3, C, U, lay, h->d_cherry, rows, rs, rlist);
  } else if (S == 64) {
    if (sc) cherry_table_kernel<64, true><<<grid, 256, 0, h->stream>>>(h->tipP, h->pmatsT, h->d_cherry3, C, U, lay, h->d_cherry, rows, rs, rlist);
    else cherry_table_kernel<64, false><<<grid, 256, 0, h->stream>>>(h->tipP, h->pmatsT, h->d_cherry3, C, U, lay, h->d_cherry, rows, rs, rlist);
  } else {
    return fail(h, PLK_ERR_UNSUPPORTED, "cherry tables for %d states", S);
  }
  HIPCHK(h, hipGetLastError());
  return PLK_OK;
}

// register levels (fragment height) of the fused program
int tree_levels(plk_handle h) {
  switch (fused_kind(h)) {
    case FK_TREE4:
      if (!jit_tree4(h)) return kTree4Levels;
      // classes in the wave: cfg5 DM 5 / 6 / 7 = 0.70 / 0.55 / 0.84 ms at G = 4
      return jit_ciw(h) ? tune_int("JIT_DM", 6, 2, 16) : tune_int("JIT_DM", 10, 2, 32);
    // jit_treeM (20 states): 4 levels (DM 3 / 4 = 3.69 / 3.43 ms on cfg3); the treeM
    // interpreter: 3 (with cherry tables 7.8 ms on cfg3, 2 levels 8.7 ms)
    case FK_TREEM:
      if (jit_treeM(h)) return tune_int("JITM_DM", 4, 2, 6);
      return 3;
    default: return 1;
  }
}

// Build the fragment programs for `ops` (validated, postorder).  Every produced node
// is emitted inside exactly one fragment; a produced internal child deeper than the
// register levels allow becomes the root of its own fragment (materialised and
// LOADed by its parent's fragment).  Fragments are grouped into tiers so that a
// fragment only reads partials written by earlier tiers.
int build_tree4_program(plk_handle h, const plk_op* ops, int n_ops, bool materialize, bool reduce) {
  const int DM = tree_levels(h);
  const int nt = h->n_tips;
  std::vector<std::vector<int> > kids(h->n_nodes);
  std::vector<char> produced(h->n_nodes, 0), is_child(h->n_nodes, 0);
  for (int i = 0; i < n_ops; ++i) {
    produced[ops[i].parent] = 1;
    for (int k = 0; k < ops[i].n_children; ++k) {
      kids[ops[i].parent].push_back(ops[i].child[k]);
      is_child[ops[i].child[k]] = 1;
    }
  }
  // produced internal children that have not been produced by an earlier op must
  // be materialised already
  std::vector<int> tops;
  for (int i = 0; i < n_ops; ++i) {
    const int n = ops[i].parent;
    if (!is_child[n] && (tops.empty() || tops.back() != n)) tops.push_back(n);
    for (int k = 0; k < ops[i].n_children; ++k) {
      const int c = ops[i].child[k];
      if (c >= nt && !produced[c] && !h->materialized[c - nt])
        return fail(h, PLK_ERR_STATE, "child %d of node %d has no partial in HBM (not computed by this call)", c,
                    n);
    }
  }
  std::sort(tops.begin(), tops.end());
  tops.erase(std::unique(tops.begin(), tops.end()), tops.end());
  // Fragments, bottom-up: the register height of a node is 1 + the largest height of
  // the produced children kept in its fragment; when that would exceed DM the
  // tallest children are cut (they become fragment roots, materialised and LOADed).
  // Cherries cost one level, so a fragment is as large a subtree as the registers
  // allow and the cut partials sit as high in the tree as possible.
  // The tree-specialised kernel also bounds the code of a fragment: a workgroup runs
  // one fragment's straight-line code, which must stay within the instruction cache,
  // so a fragment keeps at most EMAX child edges (cutting the largest kept children).
  const int EMAX = jit_tree4(h) ? 160 : (1 << 30);
  // ... and its tips' tables must fit the LDS budget (48 KiB)
  const int TMAX = jit_tree4(h) ? jit_tip_cap(h) : (1 << 30);
  // treeM: an unstored cherry (two tip children) is a leaf operand (T_CHERRY)
  std::vector<char> is_cherry(h->n_nodes, 0);
  if (!materialize && treeM_cherries(h))
    for (int n = nt; n < h->n_nodes; ++n)
      is_cherry[n] = produced[n] && is_child[n] && kids[n].size() == 2 && kids[n][0] < nt && kids[n][1] < nt;
  std::vector<int32_t> cherry3;
  std::vector<int> rh(h->n_nodes, 0), ne(h->n_nodes, 0), ntp(h->n_nodes, 0);
  std::vector<char> cut_node(h->n_nodes, 0);
  for (int i = 0; i < n_ops; ++i) {
    const int n = ops[i].parent;
    if (i + 1 < n_ops && ops[i + 1].parent == n) continue;  // polytomy: handle the node at its last op
    std::vector<int> in;
    for (int c : kids[n])
      if (c >= nt && produced[c] && !is_cherry[c]) in.push_back(c);
    std::sort(in.begin(), in.end(), [&](int x, int y) { return rh[x] > rh[y]; });
    size_t first = 0;
    while (first < in.size() && 1 + rh[in[first]] > DM) cut_node[in[first++]] = 1;
    rh[n] = 1 + (first < in.size() ? rh[in[first]] : 0);
    int edges = (int)kids[n].size(), ntips = 0;
    for (int c : kids[n]) ntips += c < nt;
    for (size_t k = first; k < in.size(); ++k) {
      edges += ne[in[k]];
      ntips += ntp[in[k]];
    }
    std::vector<int> kept(in.begin() + (long)first, in.end());
    std::sort(kept.begin(), kept.end(), [&](int x, int y) { return ne[x] > ne[y]; });
    for (size_t k = 0; k < kept.size() && (edges > EMAX || ntips > TMAX); ++k) {
      cut_node[kept[k]] = 1;
      edges -= ne[kept[k]];
      ntips -= ntp[kept[k]];
    }
    ne[n] = edges;
    ntp[n] = ntips;
    rh[n] = 1;
    for (int c : in)
      if (!cut_node[c]) rh[n] = std::max(rh[n], 1 + rh[c]);
  }
  std::vector<int> frag_of(h->n_nodes, -1);
  std::vector<int> frag_roots;
  std::vector<int> stack;
  for (int t : tops) {
    frag_of[t] = (int)frag_roots.size();
    frag_roots.push_back(t);
    stack.push_back(t);
  }
  while (!stack.empty()) {
    const int n = stack.back();
    stack.pop_back();
    for (int c : kids[n]) {
      if (c < nt || !produced[c]) continue;
      if (cut_node[c]) {
        frag_of[c] = (int)frag_roots.size();
        frag_roots.push_back(c);
      } else {
        frag_of[c] = frag_of[n];
      }
      stack.push_back(c);
    }
  }
  const int nf = (int)frag_roots.size();
  // tiers: a fragment depends on the fragments of the cut nodes it loads
  std::vector<int> tier(nf, 0);
  bool changed = true;
  while (changed) {
    changed = false;
    for (int n = nt; n < h->n_nodes; ++n) {
      if (!produced[n]) continue;
      for (int c : kids[n])
        if (c >= nt && produced[c] && frag_of[c] != frag_of[n] && tier[frag_of[n]] < tier[frag_of[c]] + 1) {
          tier[frag_of[n]] = tier[frag_of[c]] + 1;
          changed = true;
        }
    }
  }
  // emit
  std::vector<TInstr> prog;
  std::vector<int32_t> start(nf);
  const int root_reduce = (reduce && tops.size() == 1) ? tops[0] : -1;
  // node n at register level d: child events in son order, then ASCEND carrying the
  // node's own store slot and branch (the parent contributes it through that branch)
  std::function<void(int, int, bool)> emit = [&](int n, int d, bool frag_root) {
    for (int c : kids[n]) {
      if (c < nt) {
        prog.push_back({T_TIP, d, c, c});
      } else if (is_cherry[c] && frag_of[c] == frag_of[n]) {
        prog.push_back({T_CHERRY, d, (int32_t)(cherry3.size() / 3), c});
        cherry3.insert(cherry3.end(), {kids[c][0], kids[c][1], c});
      } else if (produced[c] && frag_of[c] == frag_of[n]) {
        prog.push_back({T_DESCEND, d, 0, 0});
        emit(c, d + 1, false);
      } else {
        prog.push_back({T_LOAD, d, c - nt, c});
      }
    }
    if (frag_root)
      prog.push_back({T_ASCEND, d, -1, -1});
    else
      prog.push_back({T_ASCEND, d, materialize ? n - nt : -1, n});
  };
  for (int f = 0; f < nf; ++f) {
    start[f] = (int32_t)prog.size();
    const int r = frag_roots[f];
    emit(r, 0, true);
    const bool cut = r != root_reduce && std::find(tops.begin(), tops.end(), r) == tops.end();
    prog.push_back({T_ROOT, 0, (materialize || cut) ? r - nt : -1, r == root_reduce ? 1 : 0});
  }
  // Staging chain for the LDS-staged kernel (treeM): the events that consume a table --
  // TIP (its tip table), LOAD (P^T of its branch) and a non-root ASCEND (P^T of the
  // branch its parent contributes it through) -- each carry in `d` the table of the
  // NEXT consuming event of the fragment (prefetched while the current one computes);
  // res_first[f] is the fragment's first table.  Codes: branch b >= 0 -> P^T(b), tip t
  // -> -2 - t, none -> -1.  (`d` is informational for the other kernels.)
  std::vector<int32_t> res_first(nf, -1);
  for (int f = 0; f < nf; ++f) {
    int prev = -1;
    for (size_t i = (size_t)start[f]; prog[i].op != T_ROOT; ++i) {
      TInstr& w = prog[i];
      int res;
      if (w.op == T_TIP)
        res = -2 - w.a;
      else if (w.op == T_LOAD || (w.op == T_ASCEND && w.b >= 0))
        res = w.b;
      else
        continue;
      if (prev < 0)
        res_first[f] = res;
      else
        prog[(size_t)prev].d = res;
      w.d = -1;
      prev = (int)i;
    }
  }
  int rc = ensure_cap(h, (void**)&h->d_prog, &h->d_prog_cap, prog.size() * sizeof(TInstr));
  if (rc) return rc;
  rc = ensure_cap(h, (void**)&h->d_frag, &h->d_frag_cap, 2 * std::max(nf, 1) * sizeof(int32_t));
  if (rc) return rc;
  HIPCHK(h, hipMemcpyAsync(h->d_prog, prog.data(), prog.size() * sizeof(TInstr), hipMemcpyHostToDevice, h->stream));
  // fragments sorted by tier so that each tier is a contiguous range of blockIdx.y
  std::vector<int> order(nf);
  for (int f = 0; f < nf; ++f) order[f] = f;
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return tier[x] < tier[y]; });
  std::vector<int32_t> start_sorted(2 * nf);  // [start offsets | first tables], tier order
  h->prog_tiers.clear();
  for (int i = 0; i < nf; ++i) {
    start_sorted[i] = start[order[i]];
    start_sorted[nf + i] = res_first[order[i]];
    if (h->prog_tiers.empty() || tier[order[i]] != tier[order[i - 1]]) h->prog_tiers.push_back({});
    h->prog_tiers.back().push_back(i);
  }
  HIPCHK(h, hipMemcpyAsync(h->d_frag, start_sorted.data(), 2 * nf * sizeof(int32_t), hipMemcpyHostToDevice,
                           h->stream));
  h->prog_nf = nf;
  // one counter per fragment and class (one class per workgroup, plk_jit.hpp JitShape::cls),
  // then the exit ticket
  rc = ensure_cap(h, (void**)&h->d_sbctr, &h->d_sbctr_cap, (size_t)(nf * h->C + 1) * sizeof(unsigned));
  if (rc) return rc;
  HIPCHK(h, hipMemsetAsync(h->d_sbctr, 0, (size_t)(nf * h->C + 1) * sizeof(unsigned), h->stream));
  h->prog_host = prog;
  h->frag_starts_host.assign(start_sorted.begin(), start_sorted.begin() + nf);
  h->jit_fn = nullptr;  // specialised kernel of the new program: compiled on first use
  h->jitm_fn = nullptr;
  h->jit_plan_valid = false;
  HIPCHK(h, hipStreamSynchronize(h->stream));  // host staging vectors go out of scope
  h->prog_ops.assign(ops, ops + n_ops);
  h->prog_materialize = materialize;
  h->prog_reduce = reduce;
  h->prog_dm = DM;
  h->prog_jit = jit_tree4(h);
  h->prog_jitm = jit_treeM(h);
  h->prog_ciw = jit_ciw(h);
  h->prog_tmax = TMAX;
  h->prog_root = root_reduce;
  h->cherry3.swap(cherry3);
  h->cherry_codes_valid = false;
  // bookkeeping: which partials will be in HBM after the launch (-1: untouched)
  h->prog_mat_after.assign(h->n_internal, -1);
  for (int n = nt; n < h->n_nodes; ++n)
    if (produced[n]) {
      const bool cut = frag_of[n] >= 0 && frag_roots[frag_of[n]] == n;
      h->prog_mat_after[n - nt] = (materialize || (cut && n != root_reduce)) ? 1 : 0;
      h->materialized[n - nt] = (char)h->prog_mat_after[n - nt];
    }
  return PLK_OK;
}

// the interpreter: one wave per rate class
void launch_tree4(plk_handle h, const TreeArgs& a, dim3 grid, size_t lds) {
  const dim3 block(64 * h->C);
  if (h->flags & PLK_FLAG_SCALING)
    tree4_kernel<1, kTree4Levels, true><<<grid, block, lds, h->stream>>>(a, a.prog, a.frag_start, a.pmats);
  else
    tree4_kernel<1, kTree4Levels, false><<<grid, block, lds, h->stream>>>(a, a.prog, a.frag_start, a.pmats);
}

// treeM tables: read by every wave straight from L1/L2 (no staging, no barrier) for 20
// states, staged in LDS behind one barrier per event for 64.  Measured (profiles/r01/tm1_*):
// S = 20 (16 waves per workgroup) 7.70 -> 7.48 ms direct; S = 64 (4 waves, 64x64 tables)
// 0.95 -> 1.35 ms direct.
bool treeM_direct(plk_handle h) { return h->S == 20; }

// 16-pattern groups per treeM workgroup.  20 states with direct tables: 1 (16 patterns x C
// classes, four workgroups per CU, so one workgroup's rescale barriers overlap the others'
// MFMA chains): cfg3 G = 4 / 2 / 1 = 7.40 / 6.87 / 6.43 ms (profiles/r01/g1_*); staged
// tables (64 states) need 64-pattern workgroups.
int treeM_groups(plk_handle h) { return h->S == 20 ? 1 : 4; }

// 20 states: 3 register levels, one 16-pattern group, direct tables; 64 states: 3 levels,
// four groups, staged tables
void launch_treeM(plk_handle h, const TreeArgs& a, dim3 grid, size_t lds) {
  const bool sc = (h->flags & PLK_FLAG_SCALING) != 0;
  if (h->S == 20) {
    grid.x = (unsigned)(h->n_pad / 16);
    const dim3 block(64 * h->C);
    if (sc)
      treeM_kernel<20, 3, true, true, 1><<<grid, block, lds, h->stream>>>(a, a.prog, a.frag_start, h->pmatsT);
    else
      treeM_kernel<20, 3, false, true, 1><<<grid, block, lds, h->stream>>>(a, a.prog, a.frag_start, h->pmatsT);
  } else {
    const dim3 block(64 * 4 * h->C);
    if (sc)
      treeM_kernel<64, 3, true, false, 4><<<grid, block, lds, h->stream>>>(a, a.prog, a.frag_start, h->pmatsT);
    else
      treeM_kernel<64, 3, false, false, 4><<<grid, block, lds, h->stream>>>(a, a.prog, a.frag_start, h->pmatsT);
  }
}

int update_tree4(plk_handle h, const plk_op* ops, int n_ops) {
  const bool materialize = !(h->flags & PLK_FLAG_LNL_ONLY);
  const bool reduce = h->pi_set && h->rates_set;
  const bool same = h->prog_ops.size() == (size_t)n_ops && h->prog_materialize == materialize &&
                    h->prog_reduce == reduce && h->prog_dm == tree_levels(h) && h->prog_jit == jit_tree4(h) && h->prog_ciw == jit_ciw(h) &&
                    h->prog_jitm == jit_treeM(h) &&
                    (!h->prog_jit || h->prog_tmax == jit_tip_cap(h)) &&
                    std::memcmp(h->prog_ops.data(), ops, n_ops * sizeof(plk_op)) == 0;
  if (!same) {
    int rc = build_tree4_program(h, ops, n_ops, materialize, reduce);
    if (rc) return rc;
  } else {
    for (size_t i = 0; i < h->prog_mat_after.size(); ++i)
      if (h->prog_mat_after[i] >= 0) h->materialized[i] = (char)h->prog_mat_after[i];
  }
  if (!h->table_set) return fail(h, PLK_ERR_STATE, "code table not set (plk_set_code_table)");
  const FusedKind kind = fused_kind(h);
  if (kind != FK_TREE4 || h->prog_jit) {
    int rc = refresh_tip_tables(h);
    if (rc) return rc;
  }
  if (kind == FK_TREEM) {
    int rc = ensure_pmatsT(h);
    if (rc) return rc;
    EventPair tev;
    const bool timed = (h->timing & PLK_TIME_TABLES) && !h->cherry3.empty();
    if (timed) {
      tev = get_events(h, 3);
      hipEventRecord(tev.a, h->stream);
    }
    rc = build_cherry_tables(h);
    if (rc) return rc;
    if (timed) {
      hipEventRecord(tev.b, h->stream);
      h->events.push_back(tev);
      h->n_table_launches++;
    }
  }
  TreeArgs a;
  a.uflow = h->prog_root >= 0 ? uflow_arm(h) : nullptr;
  a.cherry = h->d_cherry;
  a.prog = h->d_prog;
  a.partials = h->partials;
  a.scale = h->scale;
  a.codes = h->codes;
  a.pmats = h->pmats;
  a.init = h->code_table;
  a.tipP = h->tipP;
  a.weights = h->weights;
  a.pi = h->pi;
  a.probs = h->probs;
  a.site_lnl = h->site_lnl;
  a.wave_sums = h->wave_sums;
  a.slot_stride = h->slot_stride;
  a.n_pad = h->n_pad;
  a.n_patterns = h->n_patterns;
  a.n_codes = h->n_codes;
  a.guard = (h->flags & PLK_FLAG_NONNEG_GUARD) ? 1 : 0;
  a.n_tips = h->n_tips;
  a.C = h->C;
  a.stage_codes = (h->n_tips * 64 <= 64 * 1024) ? 1 : 0;
  const size_t lds = (size_t)((h->n_codes * 4 + 1) & ~1) * sizeof(double) + kTreeMaxWaves * 64 * sizeof(double) +
                     (a.stage_codes ? (size_t)h->n_tips * 64 : 0);
  a.n_frags = h->prog_nf;
  a.bmask = -1;
  a.cherry_pairs = 1;
  a.n_cherry_staged = 0;
  size_t lds_m = 0;
  if (kind == FK_TREEM) {
    a.buf_doubles = std::max(h->C * h->S * h->S, h->C * h->n_codes * h->S);
    a.buf_doubles = (a.buf_doubles + 1) & ~1;
    const int threads = 64 * treeM_groups(h) * (h->S == 64 ? 1 : h->C);
    const int pf = h->S == 64 ? treeM_pf<64>() : treeM_pf<20>();
    if (!h->prog_jitm && !treeM_direct(h) && a.buf_doubles > pf * threads)
      return fail(h, PLK_ERR_UNSUPPORTED, "fused MFMA tables (%d doubles) exceed the staging registers",
                  a.buf_doubles);
    a.buf_doubles = std::max(a.buf_doubles, (pf - 1) * threads);  // unconditional stores stay inside
    if (treeM_direct(h)) a.buf_doubles = 0;  // tables read from L1/L2: LDS holds the codes only
    lds_m = 2 * (size_t)a.buf_doubles * sizeof(double);
    a.stage_codes = (lds_m + (size_t)h->n_tips * 64 <= 76 * 1024) ? 1 : 0;  // two workgroups per CU
    // a program whose tips all sit in cherry tables (balanced trees) has no T_TIP event:
    // staging every tip's codes would only cost each workgroup a load of n_tips x 64 B
    if (std::none_of(h->prog_host.begin(), h->prog_host.end(), [](const TInstr& w) { return w.op == T_TIP; }))
      a.stage_codes = 0;
    if (a.stage_codes) lds_m += (size_t)h->n_tips * 64;
  }
  // 4 states, one class per wave: the tree-specialised kernel (PLK_JIT=0 keeps the
  // interpreter, e.g. for A/B measurements)
  const bool jit = h->prog_jit;
  JArgs ja;
  JitShape sh;
  if (jit) {
    sh.C = h->C;
    sh.CW = h->prog_ciw ? h->C : 1;
    sh.pin = true;  // accumulator pinning: cfg2 0.244 -> 0.241, cfg5 1.04 -> 0.93 ms
    sh.U = h->n_codes;
    sh.scale = (h->flags & PLK_FLAG_SCALING) != 0;
    // cherries read one product table (plk_jit.hpp: JitUnit) while a fragment's tables stay
    // within PLK_JIT_PAIR_KB (0: no pairs)
    const int budget = tune_int("JIT_PAIR_KB", 64, 0, 150) * 1024 / (int)sizeof(double);
    // One class per workgroup with quad units (plk_jit.hpp JitUnit, JitShape::cls): tables of
    // one class, so a fragment's cherries fit as 4-tip subtree tables -- for one class per wave,
    // no rescaling, lnL only (quads are never stored) and at most 4 codes in use (U^4 <= 256).
    // PLK_TUNE JIT_QUAD_KB bounds the tables (0: off); the plan is rebuilt as usual when it
    // gets no quad.
    const bool cls_ok = !h->prog_ciw && !sh.scale && (h->flags & PLK_FLAG_LNL_ONLY) && sh.U <= 4;
    const int qb = cls_ok ? tune_int("JIT_QUAD_KB", 136, 0, 150) * 1024 / (int)sizeof(double) : 0;
    if (!h->jit_plan_valid || h->jit_plan_U != sh.U || h->jit_plan_budget != budget || h->jit_plan_qb != qb) {
      h->jit_plan_cls = false;
      if (qb > 0) {
        h->jit_plan = jit_plan(h->prog_host, h->frag_starts_host, sh.C, sh.U, std::max(qb, budget), sh.scale, true, qb);
        for (const auto& un : h->jit_plan.units)
          for (const JitUnit& u : un) h->jit_plan_cls |= u.tc >= 0;
      }
      if (!h->jit_plan_cls) h->jit_plan = jit_plan(h->prog_host, h->frag_starts_host, sh.C, sh.U, budget, sh.scale);
      h->jit_plan_valid = true;
      h->jit_plan_U = sh.U;
      h->jit_plan_budget = budget;
      h->jit_plan_qb = qb;
      h->jit_fn = nullptr;
      h->ucodes_valid = false;
    }
    sh.cls = h->jit_plan_cls;
    if (!h->ucodes_valid) {
      std::vector<int4> units;
      for (const auto& un : h->jit_plan.units)
        for (const JitUnit& u : un) units.push_back(make_int4(u.ta, u.tb, u.tc, u.td));
      int rc = ensure_cap(h, (void**)&h->d_ucodes, &h->ucodes_cap, std::max<size_t>(units.size(), 1) * h->n_pad);
      if (!rc) rc = ensure_cap(h, (void**)&h->d_units, &h->units_cap, std::max<size_t>(units.size(), 1) * sizeof(int4));
      if (rc) return rc;
      if (!units.empty()) {
        HIPCHK(h, hipMemcpyAsync(h->d_units, units.data(), units.size() * sizeof(int4), hipMemcpyHostToDevice,
                                 h->stream));
        const dim3 ug((unsigned)((h->n_pad / 16 + 255) / 256), (unsigned)units.size());
        hipLaunchKernelGGL(unit_codes_kernel, ug, dim3(256), 0, h->stream, h->codes, h->n_pad, h->d_units, sh.U,
                           h->d_ucodes);
        HIPCHK(h, hipGetLastError());
        HIPCHK(h, hipStreamSynchronize(h->stream));  // `units` goes out of scope
      }
      h->ucodes_valid = true;
      h->ucodes_dc_valid = false;
    }
    sh.NT = h->jit_plan.NU;
    sh.TD = h->jit_plan.tab_doubles;
    sh.QT = h->jit_plan.quad_tmp;
    sh.soa = tune_int("JIT_SOA", 1, 0, 1) != 0;
    // direct codes where a fragment has at most 16 units (cfg2, 0.099 vs 0.111 ms traversal);
    // every class in the wave: up to 32 units in two 16-byte words (cfg5 shard traversal
    // 345-353 vs 367-368 us; PLK_TUNE JIT_DC_CIW=0 keeps the code rows in LDS)
    sh.dc = sh.cls ? sh.NT <= 16 && tune_int("JIT_DC", 1, 0, 1) != 0
                   : h->prog_ciw && sh.NT <= 32 && tune_int("JIT_DC_CIW", 1, 0, 1) != 0;
    sh.dcw = sh.NT <= 16 ? 1 : 2;
    if (sh.dc && (!h->ucodes_dc_valid || h->ucodes_dc_w != sh.dcw)) {
      const int nfr = (int)h->jit_plan.units.size();
      std::vector<int32_t> us(1, 0);
      for (const auto& un : h->jit_plan.units) us.push_back(us.back() + (int)un.size());
      int rc = ensure_cap(h, (void**)&h->d_ucodes_dc, &h->ucodes_dc_cap, (size_t)nfr * h->n_pad * 16 * sh.dcw);
      if (!rc) rc = ensure_cap(h, (void**)&h->d_units_start, &h->units_start_cap, us.size() * sizeof(int32_t));
      if (rc) return rc;
      HIPCHK(h, hipMemcpyAsync(h->d_units_start, us.data(), us.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                               h->stream));
      const dim3 dg((unsigned)((h->n_pad + 255) / 256), (unsigned)nfr);
      hipLaunchKernelGGL(unit_codes_dc_kernel, dg, dim3(256), 0, h->stream, h->d_ucodes, h->n_pad, h->d_units_start,
                         sh.dcw, reinterpret_cast<uint4*>(h->d_ucodes_dc));
      HIPCHK(h, hipGetLastError());
      HIPCHK(h, hipStreamSynchronize(h->stream));  // `us` goes out of scope
      h->ucodes_dc_valid = true;
      h->ucodes_dc_w = sh.dcw;
    }
    sh.ps1 = tune_int("JIT_PS1", 0, 0, 1) != 0;
    // pattern groups per workgroup (they share the staged tables): with per-node rescaling
    // and one class per wave every node has two workgroup barriers, whose cost grows with
    // the waves that meet there (cfg5: 1.93 ms at G = 2, 1.16 ms at G = 1), so one group;
    // every class in the wave (no barriers, ~230 VGPRs, two waves per SIMD): eight, the
    // whole CU's resident waves in one workgroup that stages the tables once (cfg5 at DM 6
    // with the tier's fragments side by side: G = 6 / 7 / 8 = 0.48 / 0.43 / 0.39 ms);
    // otherwise the G with the most resident waves (jit_auto_groups; cfg2 with cherry
    // tables: G = 3, 0.140 ms, G = 2 0.150, G = 4 0.162)
    // (before G: the code rows take G x PW).  With direct codes (one class per workgroup, no code
    // rows in LDS) two patterns per lane: twice the independent work per wave at four waves
    // per SIMD (cfg2 traversal 0.093 vs 0.099 ms)
    sh.PW = tune_int("JIT_PW", sh.dc && sh.cls ? 2 : 1, 1, 2);
    sh.G = tune_int("JIT_G", 0, 0, 16);
    if (sh.G == 0) {
      if (sh.cls) {
        // one class per workgroup: the tables take most of the LDS, so one workgroup per CU
        // and as many groups as fit (at most 16: 1024 threads)
        sh.G = 16;
        while (sh.G > 1 && sh.lds_bytes() > 160 * 1024 - 64) --sh.G;
      } else {
        sh.G = h->prog_ciw ? 8 : sh.scale ? 1 : jit_auto_groups(sh);
      }
    }
    sh.G = std::max(1, std::min(sh.G, 1024 / (64 * sh.nw())));  // (a JIT_G past 1024 threads)
    // two patterns per lane halve the P(t) reads per FMA but double the registers:
    // measured slower (cfg2 0.255-0.301 vs 0.241 ms), so opt-in; not with speculation
    // two-stage pipeline, codes / HBM loads 3 ahead (cfg2 0.274 -> 0.259 ms); with every
    // class in the wave a ring slot is C x larger, so there two events ahead (cfg5 0.385 ms
    // at L = 2, 0.391 at L = 1; 1.48 vs 1.04 ms at L = 3 vs 1 before the P(t) stream)
    sh.L = tune_int("JIT_L", h->prog_ciw ? 2 : 3, 1, 8);
    sh.RD = tune_int("JIT_RD", 1, 1, 8);  // table rows this many fetchers ahead (<= JIT_L)
    sh.minw = 0;
    // speculative no-rescale pass (plk_jit.hpp): a win only where rescaling never
    // fires; on cfg5 it fires in almost every super-block (1.27 vs 1.14 ms), so opt-in
    // classes in the wave: next class's P(t) loads overlap this class's FMAs
    sh.ppipe = true;
    sh.clk = env_is("PLK_DEBUG_CLOCK", '1') ? 1 : env_is("PLK_DEBUG_CLOCK", '2') ? 2 : 0;
    // PLK_JIT_BLOCKS=1: the root fragment forms the block sums (no wave_sums_to_blocks
    // launch).  Measured slower (cfg2 traversal 0.125 -> 0.160 ms): the wave that stores a
    // wave sum must wait for the store and the counter's atomic round trip (~3 us) before
    // its workgroup's next super-block barrier, in every super-block.  Off; the formal
    // release/acquire form (an L2 write-back per wave) was slower still (round 1)
    if (sh.lds_bytes() > 160 * 1024 - 64)  // (less the kernel's static LDS word)
      return fail(h, PLK_ERR_UNSUPPORTED, "tree kernel needs %zu B of LDS", sh.lds_bytes());
    if (!h->jit_fn || sh.C != h->jit_shape.C || sh.CW != h->jit_shape.CW ||
        sh.pin != h->jit_shape.pin ||
        sh.G != h->jit_shape.G || sh.U != h->jit_shape.U ||
        sh.NT != h->jit_shape.NT || sh.TD != h->jit_shape.TD || sh.scale != h->jit_shape.scale || sh.L != h->jit_shape.L ||
        sh.minw != h->jit_shape.minw || sh.ppipe != h->jit_shape.ppipe || sh.clk != h->jit_shape.clk ||
        sh.cls != h->jit_shape.cls || sh.soa != h->jit_shape.soa || sh.ps1 != h->jit_shape.ps1 || sh.RD != h->jit_shape.RD ||
        sh.dc != h->jit_shape.dc || sh.dcw != h->jit_shape.dcw) {
      int rc = jit_function(h, jit_tree4_source(h->jit_plan, sh), jit_tree4_name(sh), &h->jit_fn);
      if (rc) return rc;
      h->jit_shape = sh;
      h->jit_resident = 0;
    }
    ja.partials = a.partials;
    ja.scale = a.scale;
    ja.codes = sh.dc ? h->d_ucodes_dc : h->d_ucodes;
    ja.tipP = h->tipP;
    ja.weights = a.weights;
    ja.pi = a.pi;
    ja.probs = a.probs;
    ja.site_lnl = a.site_lnl;
    ja.wave_sums = a.wave_sums;
    ja.slot_stride = a.slot_stride;
    ja.n_pad = a.n_pad;
    ja.n_patterns = a.n_patterns;
    ja.n_sblocks = (int32_t)((h->n_pad + 64 * sh.G * sh.PW - 1) / (64 * sh.G * sh.PW));  // last may be ragged
    ja.guard = a.guard;
    ja.sb_ctr = h->d_sbctr;
    ja.dyn = tune_is("JIT_DYN", '0') ? 0 : 1;  // (per launch below)
    ja.exit_ctr = h->d_sbctr + (size_t)h->prog_nf * h->C;  // (null per launch below when not dynamic)
    ja.uflow = a.uflow;
    ja.cls_sum = nullptr;
    if (sh.cls) {
      int rc = ensure_cap(h, (void**)&h->d_cls, &h->d_cls_cap, (size_t)h->C * h->n_pad * sizeof(double));
      if (rc) return rc;
      ja.cls_sum = h->d_cls;
    }
  }
  const bool jitm = kind == FK_TREEM && h->prog_jitm;
  JMArgs ma;
  JitMShape msh;
  if (jitm) {
    msh.S = h->S;
    msh.C = h->C;
    msh.U = h->n_codes;
    msh.scale = (h->flags & PLK_FLAG_SCALING) != 0;
    msh.L = tune_int("JITM_L", 1, 1, 4);
    msh.minw = 2;
    msh.pd = 1;
    // contraction issue order: Y-outer with the A operands read ahead and pinned schedule
    // groups (plk_jitm.hpp CONTRIB; 3.77 -> 3.26 ms on cfg3); the two-stage operand fetch
    // loads the code 3 events ahead of its row
    msh.pipe = 2;
    msh.lc = 3;
    msh.G = 4;  // 16-pattern waves per workgroup (64 patterns)
    if (msh.lds_bytes() > 160 * 1024)
      return fail(h, PLK_ERR_UNSUPPORTED, "jit_treeM needs %zu B of LDS", msh.lds_bytes());
    if (!h->jitm_fn || !(msh == h->jitm_shape)) {
      int rc = jit_function(h, jit_treeM4_source(h->prog_host, h->frag_starts_host, msh), "plk_jit_treeM", &h->jitm_fn);
      if (rc) return rc;
      h->jitm_shape = msh;
    }
    const CherryLayout lay(h->C, h->n_codes, h->S, h->n_pad);
    ma.partials = h->partials;
    ma.scale = h->scale;
    ma.codes = h->codes;
    ma.tipP = h->tipP;
    ma.cherry = h->d_cherry;
    ma.pmats = h->pmats;
    ma.weights = h->weights;
    ma.pi = h->pi;
    ma.probs = h->probs;
    ma.site_lnl = h->site_lnl;
    ma.wave_sums = h->wave_sums;
    ma.slot_stride = h->slot_stride;
    ma.n_pad = h->n_pad;
    ma.n_patterns = h->n_patterns;
    ma.cherry_stride = (int64_t)lay.stride;
    ma.cherry_table_bytes = (int64_t)lay.table_bytes;
    ma.cherry_count_bytes = (int64_t)lay.count_bytes;
    ma.guard = a.guard;
    ma.uflow = a.uflow;
  }
  h->kernel_path = jit ? "jit_tree4" : jitm ? "jit_treeM" : kind == FK_TREEM ? "treeM" : "tree4";
  h->fused_cls_blocks = nullptr;
  int first = 0;
  if (jit && h->jit_shape.clk) {
    // stamp buffer for every workgroup of every tier's launch (grids below: at most
    // jit_resident workgroups per fragment of a tier)
    size_t need = 0;
    for (const auto& t : h->prog_tiers) need += (size_t)(h->n_pad / 64) * t.size() * (h->jit_shape.cls ? h->C : 1);
    if (need > h->clk_cap) {
      if (h->h_clk) hipHostFree(h->h_clk);
      h->h_clk = nullptr;
      if (hipHostMalloc((void**)&h->h_clk, need * 4 * sizeof(unsigned long long), hipHostMallocMapped) != hipSuccess ||
          hipHostGetDevicePointer((void**)&h->d_clk, h->h_clk, 0) != hipSuccess)
        return fail(h, PLK_ERR_OOM, "clock stamp buffer");
      h->clk_cap = need;
    }
    h->clk_n = 0;
  }
  for (const auto& t : h->prog_tiers) {
    a.frag_start = h->d_frag + first;
    dim3 grid((unsigned)(h->n_pad / 64), (unsigned)t.size());
    EventPair ev;
    if (h->timing & PLK_TIME_PARTIALS) {
      ev = get_events(h, 0);
      hipEventRecord(ev.a, h->stream);
    }
    if (jit) {
      const double* pm = h->pmats;
      int base = first;
      const int gz = sh.cls ? h->C : 1;  // one class per workgroup: grid.z = class
      unsigned long long* clkp = h->d_clk ? h->d_clk + 4 * h->clk_n : nullptr;
      void* args[] = {&ja, &pm, &base, &clkp};  // (the 4th only exists in a PLK_DEBUG_CLOCK build)
      // persistent grid: as many workgroups as are resident at once (occupancy query), so
      // every workgroup stages its tables once and there is no second dispatch round
      int wgs = 0;
      {
        if (h->jit_resident <= 0) {
          int per_cu = 0, n_cu = 0;
          HIPCHK(h, hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, h->jit_fn, 64 * sh.nw() * sh.G,
                                                                       sh.lds_bytes()));
          HIPCHK(h, hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, h->device));
          h->jit_resident = std::max(1, per_cu) * std::max(1, n_cu);
        }
        // every fragment of the tier at once: the resident workgroups split over the
        // fragments (each stages its fragment's tables once and walks many super-blocks)
        // instead of the tier's fragments running one after another with every workgroup
        // staging tables for a few super-blocks (cfg5 0.49 -> 0.42 ms)
        wgs = std::max(1, h->jit_resident / ((int)grid.y * gz));
      }
      const unsigned gx = (unsigned)std::min<int64_t>(ja.n_sblocks, wgs);
      // dynamic super-blocks where a workgroup walks several (a tier of 1-2 per workgroup
      // gains nothing from them and pays the counter's round trips)
      ja.dyn = (!tune_is("JIT_DYN", '0') && ja.n_sblocks >= 3 * (int64_t)gx) ? 1 : 0;
      // the launch's counters start at 0; its last workgroup leaves them at 0 (exit ticket)
      ja.exit_ctr = ja.dyn ? h->d_sbctr + (size_t)h->prog_nf * h->C : nullptr;
      h->jit_last_gx = (int)gx;
      if ((int)h->jit_frag_gx.size() < h->prog_nf) h->jit_frag_gx.resize((size_t)h->prog_nf, 0);
      for (int k = 0; k < (int)t.size(); ++k) h->jit_frag_gx[(size_t)(first + k)] = (int)gx;
      HIPCHK(h, hipModuleLaunchKernel(h->jit_fn, gx, grid.y, (unsigned)gz, 64 * sh.nw() * sh.G, 1, 1,
                                      (unsigned)sh.lds_bytes(),
                                      h->stream, args, nullptr));
      if (sh.clk) h->clk_n += (size_t)gx * grid.y * gz;
      if (sh.cls && h->prog_root >= 0 && first + (int)t.size() == h->prog_nf) {
        // the classes' root terms meet here: log, site lnL, wave and block sums (the work of
        // reduce_root and wave_sums_to_blocks), inside the traversal's timing
        h->fused_cls_blocks = block_target(h);
        launch_cls_blocks(h, ja.guard, ja.uflow, false);
      }
    } else if (jitm) {
      int base = first;
      void* args[] = {&ma, &base};
      HIPCHK(h, hipModuleLaunchKernel(h->jitm_fn, (unsigned)(h->n_pad / (16 * msh.G)), grid.y, 1,
                                      64 * msh.G, 1, 1, (unsigned)msh.lds_bytes(), h->stream, args, nullptr));
    } else if (kind == FK_TREEM) {
      launch_treeM(h, a, grid, lds_m);
      if (treeM_groups(h) != kTreeMGroups && h->prog_root >= 0 && first + (int)t.size() == h->prog_nf) {
        // 32-pattern workgroups: the root's 64-pattern wave sums from site_lnl
        site_wave_sums_kernel<<<(unsigned)(h->n_pad / 256), 256, 0, h->stream>>>(a.site_lnl, a.weights,
                                                                                 a.wave_sums, a.n_patterns, a.n_pad);
      }
    } else {
      launch_tree4(h, a, grid, lds);
    }
    HIPCHK(h, hipGetLastError());
    if (h->timing & PLK_TIME_PARTIALS) {
      hipEventRecord(ev.b, h->stream);
      h->events.push_back(ev);
    }
    if (h->timing & PLK_TIME_PARTIALS) h->n_launches++;  // launches timed by the events
    first += (int)t.size();
  }
  h->fused_lnl_valid = h->prog_root >= 0;
  h->fused_lnl_root = h->prog_root;
  // the jit kernel's root fragment formed the block sums (JitShape::blocks)
  return PLK_OK;
}

int update_levelwise(plk_handle h, const plk_op* ops, int n_ops) {
  h->kernel_path = "levelwise";
  // Validate and level the ops: level(op) = 1 + max(level of the op that last
  // wrote each internal child in this call, level of the last writer of parent).
  std::vector<int> writer_level(h->n_nodes, -1);
  std::vector<int> level(n_ops);
  int max_level = 0;
  for (int i = 0; i < n_ops; ++i) {
    const plk_op& o = ops[i];
    if (o.parent < h->n_tips || o.parent >= h->n_nodes)
      return fail(h, PLK_ERR_ARG, "op %d: parent %d is not an internal node", i, o.parent);
    if (o.n_children < 1 || o.n_children > 3) return fail(h, PLK_ERR_ARG, "op %d: %d children", i, o.n_children);
    int lv = writer_level[o.parent];
    for (int k = 0; k < o.n_children; ++k) {
      const int c = o.child[k];
      if (c < 0 || c >= h->n_nodes || c == o.parent) return fail(h, PLK_ERR_ARG, "op %d: bad child %d", i, c);
      if (!h->pmat_valid[c]) return fail(h, PLK_ERR_STATE, "op %d: transition matrix of branch %d not set", i, c);
      if (c < h->n_tips && !h->tip_set[c]) return fail(h, PLK_ERR_STATE, "op %d: tip %d has no codes", i, c);
      lv = std::max(lv, writer_level[c]);
    }
    level[i] = lv + 1;
    writer_level[o.parent] = level[i];
    max_level = std::max(max_level, level[i]);
  }
  int rc = refresh_tip_tables(h);
  if (rc) return rc;
  std::vector<int> level_start(max_level + 2, 0);
  const bool same = (int)h->last_ops.size() == n_ops &&
                    std::memcmp(h->last_ops.data(), ops, n_ops * sizeof(plk_op)) == 0;
  if (same) {
    level_start = h->last_level_start;
  } else {
  // Build device op list grouped by level (stable within a level).
  h->h_ops.clear();
  for (int i = 0; i < n_ops; ++i) level_start[level[i] + 1]++;
  for (int l = 0; l <= max_level; ++l) level_start[l + 1] += level_start[l];
  h->h_ops.resize(n_ops);
  std::vector<int> fill(level_start.begin(), level_start.end() - 1);
  for (int i = 0; i < n_ops; ++i) {
    const plk_op& o = ops[i];
    KOp k;
    std::memset(&k, 0, sizeof(k));
    k.parent = o.parent - h->n_tips;
    k.n = o.n_children;
    k.flags = o.flags;
    for (int j = 0; j < o.n_children; ++j) {
      const int c = o.child[j];
      k.branch[j] = c;
      k.is_tip[j] = c < h->n_tips;
      k.child[j] = c < h->n_tips ? c : c - h->n_tips;
    }
    h->h_ops[fill[level[i]]++] = k;
  }
  rc = ensure_cap(h, (void**)&h->d_ops, &h->d_ops_cap, n_ops * sizeof(KOp));
  if (rc) return rc;
  HIPCHK(h, hipMemcpyAsync(h->d_ops, h->h_ops.data(), n_ops * sizeof(KOp), hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));  // h_ops is pageable and reused
  h->last_ops.assign(ops, ops + n_ops);
  h->last_level_start = level_start;
  }

  PartialsArgs a;
  a.partials = h->partials;
  a.scale = h->scale;
  a.codes = h->codes;
  a.tipP = h->tipP;
  a.pmats = h->pmats;
  a.slot_stride = h->slot_stride;
  a.n_pad = h->n_pad;
  a.n_tiles = h->n_tiles;
  a.n_codes = h->n_codes;
  const bool s4 = (h->S == 4 && s4_supported(h->C) && h->n_codes <= kMaxCodes4);
  for (int l = 0; l <= max_level; ++l) {
    const int cnt = level_start[l + 1] - level_start[l];
    if (cnt == 0) continue;
    const KOp* d = h->d_ops + level_start[l];
    EventPair ev;
    if (h->timing & PLK_TIME_PARTIALS) {
      ev = get_events(h, 0);
      hipEventRecord(ev.a, h->stream);
    }
    if (s4) {
      if (h->flags & PLK_FLAG_SCALING)
        launch_s4<true>(h, d, cnt, a);
      else
        launch_s4<false>(h, d, cnt, a);
    } else {
      rc = launch_generic(h, d, cnt, a);
      if (rc) return rc;
    }
    HIPCHK(h, hipGetLastError());
    if (h->timing & PLK_TIME_PARTIALS) {
      hipEventRecord(ev.b, h->stream);
      h->events.push_back(ev);
    }
    if (h->timing & PLK_TIME_PARTIALS) h->n_launches++;  // launches timed by the events
  }
  for (int i = 0; i < n_ops; ++i) h->materialized[ops[i].parent - h->n_tips] = 1;
  h->fused_lnl_valid = false;
  h->slots_expanded = false;
  return PLK_OK;
}

// ---------------------------------------------------------------------------
// Per-subtree site-pattern compression (reference usePatterns = true,
// DRASRTreeLikelihoodData.cpp:218-332, SitePatterns P/SitePatterns.cpp:51-100).
// Bottom-up over the op list: a node's distinct patterns are the distinct tuples of its
// children's distinct-pattern ids (tips: compact codes), numbered in order of first
// appearance; its links give, per distinct pattern, each child's id.  The top node of
// the traversal stays uncompressed (every root pattern), so the root reduction and
// the per-site output are unchanged.
// ---------------------------------------------------------------------------
namespace {

// id of (a, b) pairs in order of first appearance; key space a * nb + b
struct PairIds {
  std::vector<uint64_t> keys;
  std::vector<int32_t> vals;
  uint64_t mask = 0;
  void reset(size_t n) {
    size_t cap = 16;
    while (cap < 2 * n) cap <<= 1;
    keys.assign(cap, ~0ull);
    vals.assign(cap, -1);
    mask = cap - 1;
  }
  int32_t get(uint64_t key, int32_t next) {
    uint64_t i = (key * 0x9E3779B97F4A7C15ull) >> 20 & mask;
    for (;;) {
      if (keys[i] == key) return vals[i];
      if (keys[i] == ~0ull) {
        keys[i] = key;
        vals[i] = next;
        return next;
      }
      i = (i + 1) & mask;
    }
  }
};

// ids[p] = distinct id of (a[p], b[p]); returns the number of distinct pairs
int64_t pair_ids(const int32_t* a, const int32_t* b, int64_t nb, int64_t P, std::vector<int32_t>& ids,
                 int64_t na) {
  ids.resize((size_t)P);
  int64_t D = 0;
  if ((uint64_t)na * (uint64_t)nb <= (uint64_t)4 * (uint64_t)P + 4096) {
    std::vector<int32_t> direct((size_t)(na * nb), -1);  // small key space: direct table
    for (int64_t p = 0; p < P; ++p) {
      int32_t& v = direct[(size_t)(a[p] * nb + b[p])];
      if (v < 0) v = (int32_t)D++;
      ids[(size_t)p] = v;
    }
    return D;
  }
  PairIds h;
  h.reset((size_t)P);
  for (int64_t p = 0; p < P; ++p) {
    const int32_t v = h.get((uint64_t)a[p] * (uint64_t)nb + (uint64_t)b[p], (int32_t)D);
    if (v == (int32_t)D) ++D;
    ids[(size_t)p] = v;
  }
  return D;
}

}  // namespace

int build_compression(plk_handle h, const plk_op* ops, int n_ops) {
  const int nt = h->n_tips;
  const int64_t P = h->n_patterns;
  if ((int)h->tip_codes_host.size() != nt) return fail(h, PLK_ERR_STATE, "tip codes not set");
  // logical nodes: an ACCUMULATE op continues the previous op's node
  struct LNode {
    int node;
    std::vector<int> kids;
  };
  std::vector<LNode> nodes;
  for (int i = 0; i < n_ops; ++i) {
    if ((ops[i].flags & PLK_OP_ACCUMULATE) && !nodes.empty() && nodes.back().node == ops[i].parent) {
      for (int k = 0; k < ops[i].n_children; ++k) nodes.back().kids.push_back(ops[i].child[k]);
      continue;
    }
    if (ops[i].flags & PLK_OP_ACCUMULATE)
      return fail(h, PLK_ERR_UNSUPPORTED, "pattern compression: op %d accumulates into a node of an earlier call", i);
    nodes.push_back({ops[i].parent, std::vector<int>(ops[i].child, ops[i].child + ops[i].n_children)});
  }
  std::vector<char> produced(h->n_nodes, 0), is_child(h->n_nodes, 0);
  for (const auto& n : nodes) {
    for (int c : n.kids) {
      if (c >= nt && !produced[c])
        return fail(h, PLK_ERR_STATE, "pattern compression: child %d of node %d not produced by this call", c, n.node);
      is_child[c] = 1;
    }
    produced[n.node] = 1;
  }
  h->cmp_ids.assign(h->n_internal, {});
  h->cmp_D.assign(h->n_internal, P);
  std::vector<int32_t> code32((size_t)P), tmp, tmp2;
  std::vector<std::vector<uint32_t> > node_links;  // per logical node: [k][D] concatenated
  std::vector<int64_t> nodeD(nodes.size());
  h->cmp_work = 0;
  for (size_t ni = 0; ni < nodes.size(); ++ni) {
    const LNode& n = nodes[ni];
    const int slot = n.node - nt;
    // children id arrays and counts
    std::vector<std::vector<int32_t> > kid_ids(n.kids.size());
    std::vector<const int32_t*> kid_ptr(n.kids.size());
    std::vector<int64_t> kid_D(n.kids.size());
    for (size_t k = 0; k < n.kids.size(); ++k) {
      const int c = n.kids[k];
      if (c < nt) {
        kid_ids[k].resize((size_t)P);
        const std::vector<uint8_t>& cc = h->tip_codes_host[c];
        for (int64_t p = 0; p < P; ++p) kid_ids[k][(size_t)p] = cc[(size_t)p];
        kid_ptr[k] = kid_ids[k].data();
        kid_D[k] = h->n_codes;
      } else if (h->cmp_ids[c - nt].empty()) {  // identity child (cannot happen below the top)
        kid_ids[k].resize((size_t)P);
        for (int64_t p = 0; p < P; ++p) kid_ids[k][(size_t)p] = (int32_t)p;
        kid_ptr[k] = kid_ids[k].data();
        kid_D[k] = P;
      } else {
        kid_ptr[k] = h->cmp_ids[c - nt].data();
        kid_D[k] = h->cmp_D[c - nt];
      }
    }
    int64_t D;
    std::vector<int64_t> rep;  // first pattern of each distinct id
    if (!is_child[n.node]) {
      D = P;  // top of the traversal: every root pattern
      h->cmp_ids[slot].clear();
    } else {
      std::vector<int32_t> cur(kid_ptr[0], kid_ptr[0] + P);
      int64_t Dc = kid_D[0];
      for (size_t k = 1; k < n.kids.size(); ++k) {
        Dc = pair_ids(cur.data(), kid_ptr[k], kid_D[k], P, tmp, Dc);
        cur.swap(tmp);
      }
      if (n.kids.size() == 1) {  // one child: renumber in first-appearance order
        tmp2.assign((size_t)P, 0);
        Dc = pair_ids(cur.data(), tmp2.data(), 1, P, tmp, Dc);
        cur.swap(tmp);
      }
      D = Dc;
      h->cmp_ids[slot].swap(cur);
    }
    h->cmp_D[slot] = D;
    h->cmp_work += D;
    rep.assign((size_t)D, -1);
    if (h->cmp_ids[slot].empty()) {
      for (int64_t j = 0; j < D; ++j) rep[(size_t)j] = j;
    } else {
      const std::vector<int32_t>& ids = h->cmp_ids[slot];
      for (int64_t p = 0; p < P; ++p)
        if (rep[(size_t)ids[(size_t)p]] < 0) rep[(size_t)ids[(size_t)p]] = p;
    }
    std::vector<uint32_t> lk(n.kids.size() * (size_t)D);
    for (size_t k = 0; k < n.kids.size(); ++k)
      for (int64_t j = 0; j < D; ++j) lk[k * (size_t)D + (size_t)j] = (uint32_t)kid_ptr[k][(size_t)rep[(size_t)j]];
    node_links.push_back(std::move(lk));
    nodeD[ni] = D;
  }
  // level the logical nodes and build the device op list
  std::vector<int> lev(h->n_nodes, -1), nlev(nodes.size());
  int max_level = 0;
  for (size_t ni = 0; ni < nodes.size(); ++ni) {
    int l = 0;
    for (int c : nodes[ni].kids)
      if (c >= nt) l = std::max(l, lev[c] + 1);
    lev[nodes[ni].node] = l;
    nlev[ni] = l;
    max_level = std::max(max_level, l);
  }
  std::vector<int> start(max_level + 2, 0);
  for (size_t ni = 0; ni < nodes.size(); ++ni) start[nlev[ni] + 1]++;
  for (int l = 0; l <= max_level; ++l) start[l + 1] += start[l];
  std::vector<int> fill(start.begin(), start.end() - 1);
  std::vector<KOpL> kops(nodes.size());
  std::vector<KKid> kid_recs;
  std::vector<int64_t> link_off(nodes.size());
  int64_t total = 0;
  for (size_t ni = 0; ni < nodes.size(); ++ni) {
    link_off[ni] = total;
    total += (int64_t)node_links[ni].size();
  }
  h->cmp_level_maxD.assign(max_level + 1, 0);
  for (size_t ni = 0; ni < nodes.size(); ++ni) {
    KOpL k;
    std::memset(&k, 0, sizeof(k));
    k.parent = nodes[ni].node - nt;
    k.n = (int32_t)nodes[ni].kids.size();
    k.D = (int32_t)nodeD[ni];
    k.k0 = (int32_t)kid_recs.size();
    for (int j = 0; j < k.n; ++j) {
      const int c = nodes[ni].kids[(size_t)j];
      KKid kd;
      std::memset(&kd, 0, sizeof(kd));
      kd.branch = c;
      kd.is_tip = c < nt;
      kd.child = c < nt ? c : c - nt;
      kd.link = link_off[ni] + (int64_t)j * nodeD[ni];
      kid_recs.push_back(kd);
    }
    kops[(size_t)fill[nlev[ni]]++] = k;
    h->cmp_level_maxD[nlev[ni]] = std::max<int>(h->cmp_level_maxD[nlev[ni]], k.D);
  }
  int rc = ensure_cap(h, (void**)&h->d_links, &h->d_links_cap, (size_t)std::max<int64_t>(total, 1) * sizeof(uint32_t));
  if (rc) return rc;
  rc = ensure_cap(h, (void**)&h->d_opsl, &h->d_opsl_cap, kops.size() * sizeof(KOpL));
  if (rc) return rc;
  rc = ensure_cap(h, (void**)&h->d_kidsl, &h->d_kidsl_cap, std::max<size_t>(kid_recs.size(), 1) * sizeof(KKid));
  if (rc) return rc;
  HIPCHK(h, hipMemcpy(h->d_kidsl, kid_recs.data(), kid_recs.size() * sizeof(KKid), hipMemcpyHostToDevice));
  for (size_t ni = 0; ni < nodes.size(); ++ni)
    HIPCHK(h, hipMemcpy(h->d_links + link_off[ni], node_links[ni].data(), node_links[ni].size() * sizeof(uint32_t),
                        hipMemcpyHostToDevice));
  HIPCHK(h, hipMemcpy(h->d_opsl, kops.data(), kops.size() * sizeof(KOpL), hipMemcpyHostToDevice));
  h->cmp_level_start = start;
  h->cmp_ops.assign(ops, ops + n_ops);
  h->cmp_valid = true;
  return PLK_OK;
}

template <int C>
void launch_links(plk_handle h, const KOpL* d, int cnt, int maxD, const PartialsArgs& a) {
  const dim3 grid((unsigned)((maxD + 255) / 256), (unsigned)cnt), block(256);
  if (h->flags & PLK_FLAG_SCALING)
    partials_links_s4_kernel<C, true><<<grid, block, 0, h->stream>>>(d, h->d_kidsl, a, h->d_links);
  else
    partials_links_s4_kernel<C, false><<<grid, block, 0, h->stream>>>(d, h->d_kidsl, a, h->d_links);
}

template <int S, int XB>
void launch_links_generic_S(plk_handle h, const KOpL* d, int cnt, int maxD, const PartialsArgs& a, size_t lds) {
  const dim3 grid((unsigned)((maxD + 255) / 256), (unsigned)cnt), block(256);
  if (h->flags & PLK_FLAG_SCALING)
    partials_links_generic_kernel<S, XB, true><<<grid, block, lds, h->stream>>>(d, h->d_kidsl, a, h->d_links, h->C);
  else
    partials_links_generic_kernel<S, XB, false><<<grid, block, lds, h->stream>>>(d, h->d_kidsl, a, h->d_links, h->C);
}

int launch_links_generic(plk_handle h, const KOpL* d, int cnt, int maxD, const PartialsArgs& a) {
  const size_t lds = 3 * (size_t)h->C * h->S * std::max(h->S, h->n_codes) * sizeof(double);
  if (lds > 160 * 1024) return fail(h, PLK_ERR_UNSUPPORTED, "LDS image of %zu bytes exceeds 160 KiB", lds);
  switch (h->S) {
    case 2: launch_links_generic_S<2, 2>(h, d, cnt, maxD, a, lds); break;
    case 3: launch_links_generic_S<3, 3>(h, d, cnt, maxD, a, lds); break;
    case 4: launch_links_generic_S<4, 4>(h, d, cnt, maxD, a, lds); break;
    case 20: launch_links_generic_S<20, 20>(h, d, cnt, maxD, a, lds); break;
    case 64: launch_links_generic_S<64, 16>(h, d, cnt, maxD, a, lds); break;
    default: return fail(h, PLK_ERR_UNSUPPORTED, "state count %d has no kernel instance", h->S);
  }
  return PLK_OK;
}

int update_compressed(plk_handle h, const plk_op* ops, int n_ops) {
  h->kernel_path = "subtree_patterns";
  const bool same = h->cmp_valid && h->cmp_ops.size() == (size_t)n_ops &&
                    std::memcmp(h->cmp_ops.data(), ops, n_ops * sizeof(plk_op)) == 0;
  if (!same) {
    int rc = build_compression(h, ops, n_ops);
    if (rc) return rc;
  }
  int rc = refresh_tip_tables(h);
  if (rc) return rc;
  PartialsArgs a;
  a.partials = h->partials;
  a.scale = h->scale;
  a.codes = h->codes;
  a.tipP = h->tipP;
  a.pmats = h->pmats;
  a.slot_stride = h->slot_stride;
  a.n_pad = h->n_pad;
  a.n_tiles = h->n_tiles;
  a.n_codes = h->n_codes;
  const int L = (int)h->cmp_level_start.size() - 1;
  for (int l = 0; l < L; ++l) {
    const int cnt = h->cmp_level_start[l + 1] - h->cmp_level_start[l];
    if (cnt == 0) continue;
    const KOpL* d = h->d_opsl + h->cmp_level_start[l];
    EventPair ev;
    if (h->timing & PLK_TIME_PARTIALS) {
      ev = get_events(h, 0);
      hipEventRecord(ev.a, h->stream);
    }
    const int maxD = h->cmp_level_maxD[l];
    if (h->S == 4 && s4_supported(h->C)) {
      switch (h->C) {
        case 1: launch_links<1>(h, d, cnt, maxD, a); break;
        case 2: launch_links<2>(h, d, cnt, maxD, a); break;
        case 4: launch_links<4>(h, d, cnt, maxD, a); break;
        case 8: launch_links<8>(h, d, cnt, maxD, a); break;
      }
    } else {
      int rc2 = launch_links_generic(h, d, cnt, maxD, a);
      if (rc2) return rc2;
    }
    HIPCHK(h, hipGetLastError());
    if (h->timing & PLK_TIME_PARTIALS) {
      hipEventRecord(ev.b, h->stream);
      h->events.push_back(ev);
    }
    if (h->timing & PLK_TIME_PARTIALS) h->n_launches++;  // launches timed by the events
  }
  for (int i = 0; i < n_ops; ++i) h->materialized[ops[i].parent - h->n_tips] = 1;
  h->fused_lnl_valid = false;
  h->slots_expanded = false;
  return PLK_OK;
}

// ---------------------------------------------------------------------------
// Branch derivatives for any S and C (row f1; the 4-state fast path is deriv_kernel):
// the reference's computeDownSubtreeDLikelihood / D2 twins
// (Likelihood/RHomogeneousTreeLikelihood.cpp:365-541, 615-791) as levelwise partial
// updates.  lnL is linear in the P(t) of one branch, so dL at the root is the
// traversal with P_b replaced by dP_b (d2L: d2P_b), recomputed only along the path
// from the branch to the root with every sibling read from its materialised partial.
// dP_b / d2P_b go to two scratch transition matrices (and, for a tip branch, a scratch
// tip row with its codes and table); the path vectors ping-pong between scratch slots.
// ---------------------------------------------------------------------------
int launch_partials_ops(plk_handle h, const KOp* d_ops, int n_ops) {
  PartialsArgs a;
  a.partials = h->partials;
  a.scale = h->scale;
  a.codes = h->codes;
  a.tipP = h->tipP;
  a.pmats = h->pmats;
  a.slot_stride = h->slot_stride;
  a.n_pad = h->n_pad;
  a.n_tiles = h->n_tiles;
  a.n_codes = h->n_codes;
  if (h->S == 4 && s4_supported(h->C) && h->n_codes <= kMaxCodes4) {
    if (h->flags & PLK_FLAG_SCALING)
      launch_s4<true>(h, d_ops, n_ops, a);
    else
      launch_s4<false>(h, d_ops, n_ops, a);
  } else {
    int rc = launch_generic(h, d_ops, n_ops, a);
    if (rc) return rc;
  }
  HIPCHK(h, hipGetLastError());
  return PLK_OK;
}

int materialize_last_traversal(plk_handle h);
void topo_postorder(plk_handle h, int root, std::vector<plk_op>& ops);

// plk_traversal_work: the program that served the last traversal, walked on the host.
void traversal_work(plk_handle h, plk_work* w) {
  const int S = h->S, C = h->C, nt = h->n_tips;
  const double P = (double)h->n_pad;
  std::memset(w, 0, sizeof(*w));
  w->patterns = h->n_patterns;
  // internal nodes of the last traversal and the algorithmic count
  double alg = 0.0;
  {
    std::vector<int> nk(h->n_nodes, 0), ni(h->n_nodes, 0);
    for (const plk_op& o : h->trav_ops)
      for (int k = 0; k < o.n_children; ++k) {
        nk[o.parent]++;
        if (o.child[k] >= nt) ni[o.parent]++;
      }
    for (int n = 0; n < h->n_nodes; ++n)
      if (nk[n]) {
        w->internal_nodes++;
        alg += (double)C * (2.0 * S * S * ni[n] + (double)(nk[n] - 1) * S);
      }
  }
  w->node_updates = h->n_patterns * (int64_t)w->internal_nodes;
  w->useful_flops = w->issued_flops = alg * P;
  if (h->kernel_path == "subtree_patterns") {
    w->node_updates = h->cmp_work;
    const double f = w->internal_nodes ? (double)h->cmp_work / ((double)h->n_patterns * w->internal_nodes) : 0.0;
    w->useful_flops = w->issued_flops = alg * P * f;
    return;
  }
  if (h->kernel_path == "jit_tree4" && h->jit_plan_valid) {
    // contrib: per class and state 1 mul + (S - 1) FMA, then a multiply unless it is the
    // node's first contribution (an assignment); a table row: S multiplies unless first
    double per = 0.0, tab = 0.0;
    int64_t tnodes = 0, rows = 0;
    const int U = h->n_codes;
    for (size_t f = 0; f < h->jit_plan.events.size(); ++f) {
      std::vector<char> fresh(256, 0);
      fresh[0] = 1;
      for (const JitEvent& e : h->jit_plan.events[f]) {
        const int d = e.level;
        if (e.op == T_TIP) {
          if (!fresh[d]) per += S;
          fresh[d] = 0;
        } else if (e.op == T_LOAD) {
          per += (double)S * (2 * S - 1) + (fresh[d] ? 0 : S);
          fresh[d] = 0;
        } else if (e.op == T_DESCEND) {
          fresh[d] = 1;
        } else if (e.op == T_ASCEND) {
          per += (double)S * (2 * S - 1) + (fresh[d - 1] ? 0 : S);
          fresh[d - 1] = 0;
        }
      }
      // every workgroup of the fragment builds its tables
      const int gx = f < h->jit_frag_gx.size() && h->jit_frag_gx[f] > 0 ? h->jit_frag_gx[f] : std::max(h->jit_last_gx, 1);
      for (const JitUnit& u : h->jit_plan.units[f]) {
        if (u.tb < 0) continue;
        if (u.tc >= 0) {
          // a quad replaces three nodes (two cherries and Q); per row and class: two pair
          // products, two cherry contribs, the product, Q's contrib.  With one class per
          // workgroup each of the gx x C workgroups builds its class's rows.
          tnodes += 3;
          rows += (int64_t)U * U * U * U * C;
          tab += (double)gx * C * U * U * U * U * (3.0 * S + 3.0 * S * (2 * S - 1));
          continue;
        }
        tnodes++;
        rows += (int64_t)U * U * C;
        tab += (double)gx * C * U * U * (S + (u.br >= 0 ? (double)S * (2 * S - 1) : 0.0));
      }
    }
    w->useful_flops = w->issued_flops = per * C * P;
    w->table_nodes = tnodes;
    w->table_rows = rows;
    w->table_flops = tab;
    w->node_updates = h->n_patterns * (int64_t)(w->internal_nodes - tnodes);
    w->exact = 1;
    return;
  }
  if (h->kernel_path == "jit_treeM") {
    // v_mfma_f64_4x4x4_4b: no padding rows; the first operand of a node is an assignment
    double per = 0.0;
    int64_t tnodes = 0;
    for (size_t f = 0; f < h->frag_starts_host.size(); ++f) {
      std::vector<char> fresh(64, 0);
      fresh[0] = 1;
      int d = 0;
      for (size_t i = (size_t)h->frag_starts_host[f]; h->prog_host[i].op != T_ROOT; ++i) {
        const TInstr& in = h->prog_host[i];
        if (in.op == T_TIP || in.op == T_CHERRY) {
          if (!fresh[d]) per += S;
          fresh[d] = 0;
          tnodes += in.op == T_CHERRY;
        } else if (in.op == T_LOAD) {
          per += 2.0 * S * S + (fresh[d] ? 0 : S);
          fresh[d] = 0;
        } else if (in.op == T_DESCEND) {
          fresh[++d] = 1;
        } else if (in.op == T_ASCEND && in.b >= 0) {
          per += 2.0 * S * S + (fresh[d - 1] ? 0 : S);
          fresh[--d] = 0;
        }
      }
    }
    const int nch = (int)h->cherry3.size() / 3;
    const int U = h->n_codes, XT = (S + 15) / 16, KS = S / 4;
    w->useful_flops = w->issued_flops = per * C * P;
    w->table_nodes = tnodes;
    w->table_rows = (int64_t)nch * U * U * C;
    w->table_flops = (double)nch * C * U * U * (2.0 * S * C + (double)XT * KS * 2.0 * 16 * 16 * 4 / 16);
    w->node_updates = h->n_patterns * (int64_t)(w->internal_nodes - tnodes);
    w->exact = 1;
    return;
  }
  if (h->kernel_path == "treeM") {
    // acc starts at 1 and every operand multiplies it (S per class); a contribution is an
    // MFMA chain: useful 2 S^2 per pattern and class, issued XT x KS 16x16x4 MFMAs per 16
    // patterns (32-row tiles for S = 20) plus the multiply on the padded rows
    const int XT = (S + 15) / 16, KS = S / 4;
    double use = 0.0, iss = 0.0;
    int64_t tnodes = 0;
    for (size_t i = 0; i < h->prog_host.size(); ++i) {
      const TInstr& in = h->prog_host[i];
      if (in.op == T_TIP || in.op == T_CHERRY) {
        use += S;
        iss += 16.0 * XT;
        tnodes += in.op == T_CHERRY;
      } else if (in.op == T_LOAD || (in.op == T_ASCEND && in.b >= 0)) {
        use += 2.0 * S * S + S;
        iss += (double)XT * KS * 2.0 * 16 * 16 * 4 / 16 + 16.0 * XT;
      }
    }
    const int nch = (int)h->cherry3.size() / 3;
    const int U = h->n_codes;
    w->useful_flops = use * C * P;
    w->issued_flops = iss * C * P;
    w->table_nodes = tnodes;
    w->table_rows = (int64_t)nch * U * U * C;
    // cherry_table_kernel: per cherry, class and code pair the two tip rows of every class
    // and the product through P_cherry
    w->table_flops = (double)nch * C * U * U * (2.0 * S * C + (double)XT * KS * 2.0 * 16 * 16 * 4 / 16);
    w->node_updates = h->n_patterns * (int64_t)(w->internal_nodes - tnodes);
    w->exact = 1;
    return;
  }
}

int path_derivatives(plk_handle h, int branch, double* d1, double* d2) {
  if (h->deriv_valid.empty() || !h->deriv_valid[branch])
    return fail(h, PLK_ERR_STATE, "dP/d2P of branch %d not computed (PLK_DERIV_DP | PLK_DERIV_D2P)", branch);
  if (!h->pi_set || !h->rates_set) return fail(h, PLK_ERR_STATE, "root frequencies / category rates not set");
  hipSetDevice(h->device);
  const int nt = h->n_tips;
  std::vector<std::vector<int> > kids(h->n_nodes);
  std::vector<int> parent(h->n_nodes, -1);
  // the merged tree of every traversal so far (an incremental call lists only the
  // ancestors of the changed branches)
  for (int n = 0; n < h->n_nodes; ++n)
    for (int c : h->topo_kids[n]) {
      kids[n].push_back(c);
      parent[c] = n;
    }
  if (parent[branch] < 0) return fail(h, PLK_ERR_ARG, "branch %d is not below any node of the last traversal", branch);
  int root = parent[branch];
  while (parent[root] >= 0) root = parent[root];
  // a compressed traversal's slots hold distinct subtree patterns: expand once
  bool need = !h->materialized[root - nt] || ((h->flags & PLK_FLAG_SUBTREE_PATTERNS) && !h->slots_expanded);
  for (int n = parent[branch]; n >= 0; n = parent[n])
    for (int c : kids[n])
      if (c >= nt && !h->materialized[c - nt]) need = true;
  if (need) {
    int rc = materialize_last_traversal(h);
    if (rc) return rc;
  }
  int rc = refresh_tip_tables(h);
  if (rc) return rc;
  const int C = h->C, S = h->S, nc = h->n_codes;
  const size_t PS = (size_t)C * S * S;
  const int sb[2] = {h->n_nodes, h->n_nodes + 1};     // scratch transition matrices (dP_b, d2P_b)
  const int st[2] = {nt, nt + 1};                     // scratch tip rows
  const int slot0 = h->n_internal;                    // scratch slots: pass x uses slot0 + 2x, +1
  const double* src[2] = {h->dpmats, h->d2pmats};
  for (int x = 0; x < 2; ++x) {
    HIPCHK(h, hipMemcpyAsync(h->pmats + (size_t)sb[x] * PS, src[x] + (size_t)branch * PS, PS * sizeof(double),
                             hipMemcpyDeviceToDevice, h->stream));
    if (branch < nt) {
      HIPCHK(h, hipMemcpyAsync(h->codes + (size_t)st[x] * h->n_pad, h->codes + (size_t)branch * h->n_pad,
                               (size_t)h->n_pad, hipMemcpyDeviceToDevice, h->stream));
      tip_table_kernel<<<dim3(1, C), 256, 0, h->stream>>>(h->pmats + (size_t)sb[x] * PS, h->code_table,
                                                          h->tipP + (size_t)st[x] * C * nc * S, 1, C, S, nc);
      HIPCHK(h, hipGetLastError());
    }
  }
  h->pmatsT_dirty = true;  // S = 64 kernels read the transposed copy, scratch included
  // one launch per (path node, child chunk): both passes side by side
  std::vector<std::vector<KOp> > launches;
  int path = branch, cur = 0;
  for (int n = parent[branch]; n >= 0; path = n, n = parent[n]) {
    std::vector<KOp> chunk[2];
    for (int x = 0; x < 2; ++x) {
      const int out = slot0 + 2 * x + (cur & 1), in = slot0 + 2 * x + ((cur + 1) & 1);
      const std::vector<int>& ks = kids[n];
      for (size_t k0 = 0; k0 < ks.size(); k0 += 3) {
        KOp op;
        std::memset(&op, 0, sizeof(op));
        op.parent = out;
        op.flags = k0 == 0 ? 0 : PLK_OP_ACCUMULATE;
        for (size_t k = k0; k < ks.size() && k < k0 + 3; ++k) {
          const int c = ks[k], j = op.n++;
          if (c == path && path == branch) {        // the differentiated branch
            op.is_tip[j] = c < nt;
            op.child[j] = c < nt ? st[x] : c - nt;
            op.branch[j] = sb[x];
          } else if (c == path) {                   // the path vector from the step below
            op.is_tip[j] = 0;
            op.child[j] = in;
            op.branch[j] = c;
          } else {
            op.is_tip[j] = c < nt;
            op.child[j] = c < nt ? c : c - nt;
            op.branch[j] = c;
          }
        }
        chunk[x].push_back(op);
      }
    }
    for (size_t j = 0; j < chunk[0].size(); ++j) launches.push_back({chunk[0][j], chunk[1][j]});
    ++cur;
  }
  std::vector<KOp> flat;
  for (auto& l : launches) flat.insert(flat.end(), l.begin(), l.end());
  rc = ensure_cap(h, (void**)&h->d_ops, &h->d_ops_cap, flat.size() * sizeof(KOp));
  if (rc) return rc;
  HIPCHK(h, hipMemcpyAsync(h->d_ops, flat.data(), flat.size() * sizeof(KOp), hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  h->last_ops.clear();  // d_ops now holds these ops, not the levelwise traversal's
  for (size_t l = 0; l < launches.size(); ++l) {
    rc = launch_partials_ops(h, h->d_ops + 2 * l, 2);
    if (rc) return rc;
  }
  const int last = (cur - 1) & 1;
  if (!h->d1_sums) {
    if ((rc = dalloc(h, (void**)&h->d1_sums, (size_t)(h->n_pad / 64) * sizeof(double)))) return rc;
    if ((rc = dalloc(h, (void**)&h->d2_sums, (size_t)(h->n_pad / 64) * sizeof(double)))) return rc;
  }
  DRArgs a;
  a.L = h->partials + (size_t)(root - nt) * h->slot_stride;
  a.dL = h->partials + (size_t)(slot0 + last) * h->slot_stride;
  a.d2L = h->partials + (size_t)(slot0 + 2 + last) * h->slot_stride;
  const bool sc = (h->flags & PLK_FLAG_SCALING) != 0;
  a.k0 = sc ? h->scale + (size_t)(root - nt) * h->n_pad : nullptr;
  a.k1 = sc ? h->scale + (size_t)(slot0 + last) * h->n_pad : nullptr;
  a.k2 = sc ? h->scale + (size_t)(slot0 + 2 + last) * h->n_pad : nullptr;
  a.pi = h->pi;
  a.probs = h->probs;
  a.weights = h->weights;
  a.d1_sums = h->d1_sums;
  a.d2_sums = h->d2_sums;
  a.n_patterns = h->n_patterns;
  a.S = S;
  a.C = C;
  a.guard = (h->flags & PLK_FLAG_NONNEG_GUARD) ? 1 : 0;
  deriv_reduce_kernel<<<(unsigned)(h->n_pad / 256), 256, 0, h->stream>>>(a);
  HIPCHK(h, hipGetLastError());
  const int n_waves = (int)((h->n_patterns + 63) / 64);
  std::vector<double> w1(n_waves), w2(n_waves);
  HIPCHK(h, hipMemcpyAsync(w1.data(), h->d1_sums, n_waves * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipMemcpyAsync(w2.data(), h->d2_sums, n_waves * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  double s1 = 0.0, s2 = 0.0;
  for (int i = 0; i < n_waves; ++i) {
    s1 += w1[i];
    s2 += w2[i];
  }
  if (d1) *d1 = s1;
  if (d2) *d2 = s2;
  return PLK_OK;
}

// plk_root_pair_derivatives: the five root products with dP / d2P substituted on the two
// root sons a and b (scratch matrices and, for tip sons, scratch tip rows), formed by the
// levelwise partial kernels into scratch slots, then pair_reduce_kernel (plk_deriv.hpp).
int root_pair_derivatives(plk_handle h, int a, int b, double alpha, double beta, double* d1, double* d2) {
  if (a == b || a < 0 || b < 0 || a >= h->n_nodes || b >= h->n_nodes)
    return fail(h, PLK_ERR_ARG, "bad root sons %d, %d", a, b);
  for (int x : {a, b})
    if (h->deriv_valid.empty() || !h->deriv_valid[x])
      return fail(h, PLK_ERR_STATE, "dP/d2P of branch %d not computed (PLK_DERIV_DP | PLK_DERIV_D2P)", x);
  if (!h->pi_set || !h->rates_set) return fail(h, PLK_ERR_STATE, "root frequencies / category rates not set");
  if (h->trav_ops.empty()) return fail(h, PLK_ERR_STATE, "no traversal yet (plk_update_partials)");
  hipSetDevice(h->device);
  const int nt = h->n_tips;
  std::vector<int> parent(h->n_nodes, -1);
  for (int n = 0; n < h->n_nodes; ++n)
    for (int c : h->topo_kids[n]) parent[c] = n;
  const int root = parent[a];
  if (root < 0 || parent[b] != root || parent[root] >= 0)
    return fail(h, PLK_ERR_ARG, "branches %d and %d are not both sons of the traversal's root", a, b);
  const std::vector<int>& ks = h->topo_kids[root];
  bool need = !h->materialized[root - nt] || ((h->flags & PLK_FLAG_SUBTREE_PATTERNS) && !h->slots_expanded);
  for (int c : ks)
    if (c >= nt && !h->materialized[c - nt]) need = true;
  int rc;
  if (need && (rc = materialize_last_traversal(h))) return rc;
  if ((rc = refresh_tip_tables(h))) return rc;
  const int C = h->C, S = h->S, nc = h->n_codes;
  const size_t PS = (size_t)C * S * S;
  // scratch matrices / tip rows: 0 dP_a, 1 d2P_a, 2 dP_b, 3 d2P_b
  const int son[4] = {a, a, b, b};
  const double* src[4] = {h->dpmats, h->d2pmats, h->dpmats, h->d2pmats};
  for (int x = 0; x < 4; ++x) {
    const int sm = h->n_nodes + x, st = nt + x;
    HIPCHK(h, hipMemcpyAsync(h->pmats + (size_t)sm * PS, src[x] + (size_t)son[x] * PS, PS * sizeof(double),
                             hipMemcpyDeviceToDevice, h->stream));
    if (son[x] < nt) {
      HIPCHK(h, hipMemcpyAsync(h->codes + (size_t)st * h->n_pad, h->codes + (size_t)son[x] * h->n_pad,
                               (size_t)h->n_pad, hipMemcpyDeviceToDevice, h->stream));
      tip_table_kernel<<<dim3(1, C), 256, 0, h->stream>>>(h->pmats + (size_t)sm * PS, h->code_table,
                                                          h->tipP + (size_t)st * C * nc * S, 1, C, S, nc);
      HIPCHK(h, hipGetLastError());
    }
  }
  h->pmatsT_dirty = true;
  // variant v: scratch index substituted on a and on b (-1 = the son's own P)
  const int sub[5][2] = {{0, -1}, {-1, 2}, {1, -1}, {-1, 3}, {0, 2}};
  const int slot0 = h->n_internal;
  std::vector<KOp> flat;
  const size_t n_chunks = (ks.size() + 2) / 3;
  for (size_t k0 = 0; k0 < ks.size(); k0 += 3)
    for (int v = 0; v < 5; ++v) {
      KOp op;
      std::memset(&op, 0, sizeof(op));
      op.parent = slot0 + v;
      op.flags = k0 == 0 ? 0 : PLK_OP_ACCUMULATE;
      for (size_t k = k0; k < ks.size() && k < k0 + 3; ++k) {
        const int c = ks[k], j = op.n++;
        const int x = c == a ? sub[v][0] : c == b ? sub[v][1] : -1;
        op.is_tip[j] = c < nt;
        op.child[j] = c < nt ? (x >= 0 ? nt + x : c) : c - nt;
        op.branch[j] = x >= 0 ? h->n_nodes + x : c;
      }
      flat.push_back(op);
    }
  if ((rc = ensure_cap(h, (void**)&h->d_ops, &h->d_ops_cap, flat.size() * sizeof(KOp)))) return rc;
  HIPCHK(h, hipMemcpyAsync(h->d_ops, flat.data(), flat.size() * sizeof(KOp), hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  h->last_ops.clear();  // d_ops now holds these ops, not the levelwise traversal's
  for (size_t l = 0; l < n_chunks; ++l)
    if ((rc = launch_partials_ops(h, h->d_ops + 5 * l, 5))) return rc;
  if (!h->d1_sums) {
    if ((rc = dalloc(h, (void**)&h->d1_sums, (size_t)(h->n_pad / 64) * sizeof(double)))) return rc;
    if ((rc = dalloc(h, (void**)&h->d2_sums, (size_t)(h->n_pad / 64) * sizeof(double)))) return rc;
  }
  const bool sc = (h->flags & PLK_FLAG_SCALING) != 0;
  PairArgs pa;
  pa.L = h->partials + (size_t)(root - nt) * h->slot_stride;
  pa.k0 = sc ? h->scale + (size_t)(root - nt) * h->n_pad : nullptr;
  for (int v = 0; v < 5; ++v) {
    pa.X[v] = h->partials + (size_t)(slot0 + v) * h->slot_stride;
    pa.kx[v] = sc ? h->scale + (size_t)(slot0 + v) * h->n_pad : nullptr;
  }
  pa.pi = h->pi;
  pa.probs = h->probs;
  pa.weights = h->weights;
  pa.d1_sums = h->d1_sums;
  pa.d2_sums = h->d2_sums;
  pa.n_patterns = h->n_patterns;
  pa.alpha = alpha;
  pa.beta = beta;
  pa.S = S;
  pa.C = C;
  pa.guard = (h->flags & PLK_FLAG_NONNEG_GUARD) ? 1 : 0;
  pair_reduce_kernel<<<(unsigned)(h->n_pad / 256), 256, 0, h->stream>>>(pa);
  HIPCHK(h, hipGetLastError());
  const int n_waves = (int)((h->n_patterns + 63) / 64);
  std::vector<double> w1(n_waves), w2(n_waves);
  HIPCHK(h, hipMemcpyAsync(w1.data(), h->d1_sums, n_waves * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipMemcpyAsync(w2.data(), h->d2_sums, n_waves * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  double s1 = 0.0, s2 = 0.0;
  for (int i = 0; i < n_waves; ++i) {
    s1 += w1[i];
    s2 += w2[i];
  }
  if (d1) *d1 = s1;
  if (d2) *d2 = s2;
  return PLK_OK;
}

int validate_ops(plk_handle h, const plk_op* ops, int n_ops) {
  std::vector<char> done(h->n_nodes, 0);
  for (int i = 0; i < n_ops; ++i) {
    const plk_op& o = ops[i];
    if (o.parent < h->n_tips || o.parent >= h->n_nodes)
      return fail(h, PLK_ERR_ARG, "op %d: parent %d is not an internal node", i, o.parent);
    if (o.n_children < 1 || o.n_children > 3) return fail(h, PLK_ERR_ARG, "op %d: %d children", i, o.n_children);
    if ((o.flags & PLK_OP_ACCUMULATE) && !done[o.parent] && !h->materialized[o.parent - h->n_tips])
      return fail(h, PLK_ERR_STATE, "op %d: accumulate into node %d that has no partial", i, o.parent);
    for (int k = 0; k < o.n_children; ++k) {
      const int c = o.child[k];
      if (c < 0 || c >= h->n_nodes || c == o.parent) return fail(h, PLK_ERR_ARG, "op %d: bad child %d", i, c);
      if (!h->pmat_valid[c]) return fail(h, PLK_ERR_STATE, "op %d: transition matrix of branch %d not set", i, c);
      if (c < h->n_tips && !h->tip_set[c]) return fail(h, PLK_ERR_STATE, "op %d: tip %d has no codes", i, c);
    }
    done[o.parent] = 1;
  }
  return PLK_OK;
}

// An op list is fusable when every ACCUMULATE op continues the node of the op
// just before it (the polytomy split produced by the host) -- then the program
// treats the node as one multi-child node.
bool fusable(const plk_op* ops, int n_ops) {
  for (int i = 0; i < n_ops; ++i)
    if ((ops[i].flags & PLK_OP_ACCUMULATE) && (i == 0 || ops[i - 1].parent != ops[i].parent)) return false;
  return true;
}

// Re-run the traversal of the whole (merged) tree writing every partial (same arithmetic,
// identical values).
int materialize_last_traversal(plk_handle h) {
  std::vector<int> parent(h->n_nodes, -1);
  for (int n = 0; n < h->n_nodes; ++n)
    for (int c : h->topo_kids[n]) parent[c] = n;
  int root = h->trav_ops.back().parent;
  while (parent[root] >= 0) root = parent[root];
  std::vector<plk_op> ops;
  topo_postorder(h, root, ops);
  const unsigned saved = h->flags;
  h->flags &= ~(unsigned)PLK_FLAG_LNL_ONLY;
  const int rc = tree4_supported(h) && fusable(ops.data(), (int)ops.size())
                     ? update_tree4(h, ops.data(), (int)ops.size())
                     : update_levelwise(h, ops.data(), (int)ops.size());
  h->flags = saved;
  if (!rc && (h->flags & PLK_FLAG_SUBTREE_PATTERNS)) h->slots_expanded = true;
  return rc;
}

// Postorder op list of the merged topology below `root` (<= 3 children per op; a
// polytomy continues with ACCUMULATE ops), as the host would hand it over.
void topo_postorder(plk_handle h, int root, std::vector<plk_op>& ops) {
  std::vector<std::pair<int, size_t> > st(1, std::make_pair(root, (size_t)0));
  while (!st.empty()) {
    const int n = st.back().first;
    const std::vector<int>& ks = h->topo_kids[n];
    if (st.back().second < ks.size()) {
      const int c = ks[st.back().second++];
      if (c >= h->n_tips) st.push_back(std::make_pair(c, (size_t)0));
      continue;
    }
    for (size_t k0 = 0; k0 < ks.size(); k0 += 3) {
      plk_op o;
      std::memset(&o, 0, sizeof(o));
      o.parent = n;
      o.flags = k0 == 0 ? 0 : PLK_OP_ACCUMULATE;
      for (size_t k = k0; k < ks.size() && k < k0 + 3; ++k) o.child[o.n_children++] = ks[k];
      ops.push_back(o);
    }
    st.pop_back();
  }
}

// ---------------------------------------------------------------------------
// Double-recursive derivatives of every branch (plk_dr.hpp; row f4):
// DRHomogeneousTreeLikelihood::computeSubtreeLikelihoodPrefix (:543-651) as a
// levelwise preorder pass of ordinary partial updates into the U slots, then one
// reduction launch over all branches (computeTreeDLikelihoods / D2 twins :287-423).
// ---------------------------------------------------------------------------
// Row f4 for 4 states without rescaling: dr_pre_s4_kernel level by level (fathers of
// depth d in one launch), then the fixed-order sums of the per-block branch terms.
int dr_fused_preorder(plk_handle h, const std::vector<std::vector<int> >& depth, const std::vector<int>& parent,
                      int root, double* d1, double* d2) {
  const int C = h->C, nt = h->n_tips, nn = h->n_nodes;
  (void)parent;
  std::vector<DrBranch> br;  // one row per branch (dr_sum_kernel's node map)
  std::vector<int> bidx(nn, -1);
  for (size_t d = 1; d < depth.size(); ++d)
    for (int v : depth[d]) {
      DrBranch b;
      std::memset(&b, 0, sizeof(b));
      b.node = v;
      bidx[v] = (int)br.size();
      br.push_back(b);
    }
  std::vector<DrPreOp> ops;
  struct Level {
    size_t first;
    int count;
    int ns;  // 2: every father of the launch has <= 2 sons (the MFMA kernels' NS)
  };
  std::vector<Level> levels;
  for (size_t d = 0; d + 1 < depth.size(); ++d)
    for (int ns = 2; ns <= 3; ++ns) {  // fathers of <= 2 sons first, then the others
      const size_t first = ops.size();
      for (int f : depth[d]) {
        if (f < nt) continue;
        if (((int)h->topo_kids[f].size() <= 2) != (ns == 2)) continue;
        DrPreOp op;
        std::memset(&op, 0, sizeof(op));
        op.f = f;
        op.uf_slot = f == root ? -1 : h->dr_slot0 + f;
        for (int v : h->topo_kids[f]) {
          const int j = op.n++;
          op.son[j] = v;
          op.is_tip[j] = v < nt;
          op.idx[j] = v < nt ? v : v - nt;
          op.uslot[j] = v < nt ? -1 : h->dr_slot0 + v;
          op.bidx[j] = bidx[v];
        }
        ops.push_back(op);
      }
      if (ops.size() > first) levels.push_back(Level{first, (int)(ops.size() - first), ns});
    }
  const bool mfma = h->S == 20;
  const bool sc = (h->flags & PLK_FLAG_SCALING) != 0;
  const int n_blk = (int)(h->n_pad / (mfma ? 64 : kDrThreads));
  int rc;
  if ((rc = ensure_cap(h, (void**)&h->d_drb, &h->d_drb_cap, br.size() * sizeof(DrBranch)))) return rc;
  if ((rc = ensure_cap(h, (void**)&h->d_drpre, &h->d_drpre_cap, ops.size() * sizeof(DrPreOp)))) return rc;
  if ((rc = ensure_cap(h, (void**)&h->dr_blk, &h->dr_blk_cap, 2 * br.size() * n_blk * sizeof(double)))) return rc;
  if (!h->dr_out && (rc = dalloc(h, (void**)&h->dr_out, 2 * (size_t)nn * sizeof(double)))) return rc;
  HIPCHK(h, hipMemcpyAsync(h->d_drb, br.data(), br.size() * sizeof(DrBranch), hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipMemcpyAsync(h->d_drpre, ops.data(), ops.size() * sizeof(DrPreOp), hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipMemsetAsync(h->dr_out, 0, 2 * (size_t)nn * sizeof(double), h->stream));
  DrArgs a;
  std::memset(&a, 0, sizeof(a));
  a.partials = h->partials;
  a.codes = h->codes;
  a.code_table = h->code_table;
  a.pmats = h->pmats;
  a.dpmats = h->dpmats;
  a.d2pmats = h->d2pmats;
  a.pi = h->pi;
  a.probs = h->probs;
  a.weights = h->weights;
  a.tipP = h->tipP;
  a.n_codes = h->n_codes;
  a.blk1 = h->dr_blk;
  a.blk2 = h->dr_blk + br.size() * n_blk;
  a.slot_stride = h->slot_stride;
  a.n_pad = h->n_pad;
  a.n_patterns = h->n_patterns;
  a.C = C;
  a.n_blk = n_blk;
  a.uout = h->partials;
  EventPair ev;
  if (h->timing & PLK_TIME_PARTIALS) {
    ev = get_events(h, 0);
    hipEventRecord(ev.a, h->stream);
  }
  for (const Level& l : levels) {
    const dim3 grid((unsigned)n_blk, (unsigned)l.count);
    const DrPreOp* o = h->d_drpre + l.first;
    if (mfma) {  // 20 states: 4x4x4 matrix-core tiles, no padding (plk_dr.hpp: dr_pre_m20_kernel)
#define PLK_DRM20_NS(C_, NS_)                                                                 \
  (sc ? dr_pre_m20_kernel<C_, true, NS_><<<grid, 256, 0, h->stream>>>(o, a)                  \
      : dr_pre_m20_kernel<C_, false, NS_><<<grid, 256, 0, h->stream>>>(o, a))
#define PLK_DRM20(C_) (l.ns == 2 ? PLK_DRM20_NS(C_, 2) : PLK_DRM20_NS(C_, 3))
      switch (C) {
        case 1: PLK_DRM20(1); break;
        case 2: PLK_DRM20(2); break;
        case 4: PLK_DRM20(4); break;
      }
#undef PLK_DRM20
#undef PLK_DRM20_NS
    } else if (sc) {
      switch (C) {
        case 1: dr_pre_s4_kernel<1, true><<<grid, kDrThreads, 0, h->stream>>>(o, a, h->partials, h->partials); break;
        case 2: dr_pre_s4_kernel<2, true><<<grid, kDrThreads, 0, h->stream>>>(o, a, h->partials, h->partials); break;
        case 4: dr_pre_s4_kernel<4, true><<<grid, kDrThreads, 0, h->stream>>>(o, a, h->partials, h->partials); break;
      }
    } else {
      switch (C) {
        case 1: dr_pre_s4_kernel<1><<<grid, kDrThreads, 0, h->stream>>>(o, a, h->partials, h->partials); break;
        case 2: dr_pre_s4_kernel<2><<<grid, kDrThreads, 0, h->stream>>>(o, a, h->partials, h->partials); break;
        case 4: dr_pre_s4_kernel<4><<<grid, kDrThreads, 0, h->stream>>>(o, a, h->partials, h->partials); break;
      }
    }
    HIPCHK(h, hipGetLastError());
  }
  if (h->timing & PLK_TIME_PARTIALS) {
    hipEventRecord(ev.b, h->stream);
    h->events.push_back(ev);
  }
  dr_sum_kernel<<<(unsigned)br.size(), 256, 0, h->stream>>>(h->d_drb, a.blk1, a.blk2, n_blk, h->dr_out, h->dr_out + nn);
  HIPCHK(h, hipGetLastError());
  std::vector<double> out(2 * (size_t)nn);
  HIPCHK(h, hipMemcpyAsync(out.data(), h->dr_out, out.size() * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  if (d1) std::copy(out.begin(), out.begin() + nn, d1);
  if (d2) std::copy(out.begin() + nn, out.end(), d2);
  return PLK_OK;
}

int dr_derivatives(plk_handle h, double* d1, double* d2) {
  if (!(h->flags & PLK_FLAG_DOUBLE_RECURSIVE))
    return fail(h, PLK_ERR_STATE, "handle was not created with PLK_FLAG_DOUBLE_RECURSIVE");
  if (h->trav_ops.empty()) return fail(h, PLK_ERR_STATE, "no traversal yet (plk_update_partials)");
  if (!h->pi_set || !h->rates_set) return fail(h, PLK_ERR_STATE, "root frequencies / category rates not set");
  const int S = h->S, C = h->C, nt = h->n_tips, nn = h->n_nodes;
  if (!(S == 2 || S == 3 || S == 4 || S == 20 || S == 64))
    return fail(h, PLK_ERR_UNSUPPORTED, "state count %d has no kernel instance", S);
  hipSetDevice(h->device);
  std::vector<int> parent(nn, -1);
  for (int n = 0; n < nn; ++n)
    for (int c : h->topo_kids[n]) parent[c] = n;
  int root = h->trav_ops.back().parent;
  while (parent[root] >= 0) root = parent[root];
  if (h->topo_kids[root].size() < 2) return fail(h, PLK_ERR_UNSUPPORTED, "root %d has fewer than two sons", root);
  // preorder levels (depth 1 = sons of the root)
  std::vector<std::vector<int> > depth(1, std::vector<int>(1, root));
  while (true) {
    std::vector<int> next;
    for (int n : depth.back())
      for (int c : h->topo_kids[n]) next.push_back(c);
    if (next.empty()) break;
    depth.push_back(next);
  }
  bool need = false;
  for (size_t d = 0; d < depth.size(); ++d)
    for (int v : depth[d]) {
      if (d > 0 && (h->deriv_valid.empty() || !h->deriv_valid[v]))
        return fail(h, PLK_ERR_STATE, "dP/d2P of branch %d not computed (PLK_DERIV_DP | PLK_DERIV_D2P)", v);
      if (v >= nt && !h->materialized[v - nt]) need = true;
    }
  int rc;
  if (need) {  // every L_v is read from HBM: materialise the whole tree once
    std::vector<plk_op> ops;
    topo_postorder(h, root, ops);
    const unsigned saved = h->flags;
    h->flags &= ~(unsigned)PLK_FLAG_LNL_ONLY;
    rc = tree4_supported(h) && fusable(ops.data(), (int)ops.size()) ? update_tree4(h, ops.data(), (int)ops.size())
                                                                    : update_levelwise(h, ops.data(), (int)ops.size());
    h->flags = saved;
    if (rc) return rc;
  }
  if ((rc = refresh_tip_tables(h))) return rc;
  if ((S == 20 || S == 64) && (rc = ensure_pmatsT(h))) return rc;
  // 4 and 20 states (1, 2 or 4 classes, any rescaling): the fused preorder
  // (dr_pre_s4_kernel / dr_pre_m20_kernel), one launch per level of fathers, branch terms
  // reduced where U is formed.  Otherwise (64 states, other class counts, fathers of more
  // than three sons) the levelwise preorder + reduction below: a fused 64-state preorder on
  // 16x16x4 tiles held 342 registers (one wave per SIMD) and ran cfg4's pass in 17.7 ms
  // against 12.7 ms levelwise (profiles/r03/r3e), so it was removed
  bool pre = (S == 4 || S == 20) && (C == 1 || C == 2 || C == 4);
  for (size_t d = 0; pre && d < depth.size(); ++d)
    for (int f : depth[d])
      if (f >= nt && (h->topo_kids[f].size() < 2 || h->topo_kids[f].size() > 3)) pre = false;
  if (pre) return dr_fused_preorder(h, depth, parent, root, d1, d2);
  // M_f for every internal father below the root
  std::vector<int2> mlist;
  for (size_t d = 1; d < depth.size(); ++d)
    for (int f : depth[d])
      if (f >= nt && !h->topo_kids[f].empty()) mlist.push_back(make_int2(f, parent[f] == root ? 1 : 0));
  const int mat_base = nn + kScratchMats;
  if (!mlist.empty()) {
    if ((rc = ensure_cap(h, (void**)&h->d_drm, &h->d_drm_cap, mlist.size() * sizeof(int2)))) return rc;
    HIPCHK(h, hipMemcpyAsync(h->d_drm, mlist.data(), mlist.size() * sizeof(int2), hipMemcpyHostToDevice, h->stream));
    dr_matrix_kernel<<<dim3((unsigned)mlist.size(), C), 256, 0, h->stream>>>(
        h->pmats, h->pmats, (S == 20 || S == 64) ? h->pmatsT : nullptr, h->pi, h->d_drm, mat_base, C, S);
    HIPCHK(h, hipGetLastError());
  }
  // S = 20 / 64 reduce on fp64 MFMA (64-pattern blocks)
  const bool dr_mfma = S == 20 || S == 64;
  // tips whose father has one other son and a father of its own: U_v formed inside the
  // reduction (S <= 4 kernel), never stored
  std::vector<char> fused(nn, 0);
  if (!dr_mfma && S <= 4)
    for (int v = 0; v < nt; ++v)
      if (parent[v] >= 0 && parent[v] != root && h->topo_kids[parent[v]].size() == 2) fused[v] = 1;
  // U_v for every non-root node, one launch per (depth, child chunk)
  std::vector<KOp> flat;
  std::vector<std::pair<size_t, int> > launches;
  for (size_t d = 1; d < depth.size(); ++d) {
    std::vector<std::vector<KOp> > chunks;
    for (int v : depth[d]) {
      if (fused[v]) continue;
      const int f = parent[v];
      std::vector<int> ck_tip, ck_child, ck_branch;
      if (f != root) {
        ck_tip.push_back(0);
        ck_child.push_back(h->dr_slot0 + f);
        ck_branch.push_back(mat_base + f);
      }
      for (int s : h->topo_kids[f])
        if (s != v) {
          ck_tip.push_back(s < nt);
          ck_child.push_back(s < nt ? s : s - nt);
          ck_branch.push_back(s);
        }
      for (size_t k0 = 0, j = 0; k0 < ck_tip.size(); k0 += 3, ++j) {
        KOp op;
        std::memset(&op, 0, sizeof(op));
        op.parent = h->dr_slot0 + v;
        op.flags = k0 == 0 ? 0 : PLK_OP_ACCUMULATE;
        for (size_t k = k0; k < ck_tip.size() && k < k0 + 3; ++k) {
          const int i = op.n++;
          op.is_tip[i] = ck_tip[k];
          op.child[i] = ck_child[k];
          op.branch[i] = ck_branch[k];
        }
        if (chunks.size() <= j) chunks.resize(j + 1);
        chunks[j].push_back(op);
      }
    }
    for (auto& ch : chunks) {
      launches.push_back(std::make_pair(flat.size(), (int)ch.size()));
      flat.insert(flat.end(), ch.begin(), ch.end());
    }
  }
  if ((rc = ensure_cap(h, (void**)&h->d_ops, &h->d_ops_cap, flat.size() * sizeof(KOp)))) return rc;
  HIPCHK(h, hipMemcpyAsync(h->d_ops, flat.data(), flat.size() * sizeof(KOp), hipMemcpyHostToDevice, h->stream));
  h->last_ops.clear();  // d_ops now holds the preorder ops
  for (auto& l : launches)
    if ((rc = launch_partials_ops(h, h->d_ops + l.first, l.second))) return rc;
  // all branches in one reduction launch
  std::vector<DrBranch> br;
  for (size_t d = 1; d < depth.size(); ++d)
    for (int v : depth[d]) {
      DrBranch b;
      std::memset(&b, 0, sizeof(b));
      b.node = v;
      b.is_tip = v < nt;
      b.child = v < nt ? v : v - nt;
      b.uslot = h->dr_slot0 + v;
      b.use_pi = parent[v] == root;
      if (fused[v]) {
        const int f = parent[v];
        const int sb = h->topo_kids[f][0] == v ? h->topo_kids[f][1] : h->topo_kids[f][0];
        b.fuse = 1;
        b.uf_slot = h->dr_slot0 + f;
        b.mf = mat_base + f;
        b.sib_tip = sb < nt;
        b.sib = sb < nt ? sb : sb - nt;
        b.sib_branch = sb;
      }
      br.push_back(b);
    }
  const int n_blk = (int)(h->n_pad / (dr_mfma ? 64 : kDrThreads));
  if ((rc = ensure_cap(h, (void**)&h->d_drb, &h->d_drb_cap, br.size() * sizeof(DrBranch)))) return rc;
  if ((rc = ensure_cap(h, (void**)&h->dr_blk, &h->dr_blk_cap, 2 * br.size() * n_blk * sizeof(double)))) return rc;
  if (!h->dr_out && (rc = dalloc(h, (void**)&h->dr_out, 2 * (size_t)nn * sizeof(double)))) return rc;
  HIPCHK(h, hipMemcpyAsync(h->d_drb, br.data(), br.size() * sizeof(DrBranch), hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipMemsetAsync(h->dr_out, 0, 2 * (size_t)nn * sizeof(double), h->stream));
  DrArgs a;
  a.partials = h->partials;
  a.codes = h->codes;
  a.code_table = h->code_table;
  a.pmats = h->pmats;
  a.dpmats = h->dpmats;
  a.d2pmats = h->d2pmats;
  a.pi = h->pi;
  a.probs = h->probs;
  a.weights = h->weights;
  a.tipP = h->tipP;
  a.n_codes = h->n_codes;
  a.blk1 = h->dr_blk;
  a.blk2 = h->dr_blk + br.size() * n_blk;
  a.slot_stride = h->slot_stride;
  a.n_pad = h->n_pad;
  a.n_patterns = h->n_patterns;
  a.C = C;
  a.n_blk = n_blk;
  a.G = 3 * (size_t)C * S * S * sizeof(double) <= 96 * 1024 ? C : 1;
  dim3 grid((unsigned)n_blk, (unsigned)br.size());
  const size_t lds = 3 * (size_t)a.G * S * S * sizeof(double);
  EventPair ev;
  if (h->timing & PLK_TIME_PARTIALS) {
    ev = get_events(h, 0);
    hipEventRecord(ev.a, h->stream);
  }
  if (dr_mfma) {
    DrArgs am = a;
    am.G = 3 * (size_t)C * S * S * sizeof(double) <= 64 * 1024 ? C : 1;
    const size_t lds_m = 3 * (size_t)am.G * S * S * sizeof(double);
    // a few workgroups per branch, each looping over pattern blocks (4096 in total)
    constexpr int want = 4096;
    grid.x = (unsigned)std::min<int64_t>(n_blk, std::max<int64_t>(1, (want + (int)br.size() - 1) / (int)br.size()));
    if (S == 20)
      dr_branch_mfma_kernel<20><<<grid, kDrmThreads, lds_m, h->stream>>>(h->d_drb, am);
    else
      dr_branch_mfma_kernel<64><<<grid, kDrmThreads, lds_m, h->stream>>>(h->d_drb, am);
  } else {
    switch (S) {
      case 2: dr_branch_kernel<2><<<grid, kDrThreads, lds, h->stream>>>(h->d_drb, a); break;
      case 3: dr_branch_kernel<3><<<grid, kDrThreads, lds, h->stream>>>(h->d_drb, a); break;
      case 4: dr_branch_kernel<4><<<grid, kDrThreads, lds, h->stream>>>(h->d_drb, a); break;
    }
  }
  HIPCHK(h, hipGetLastError());
  if (h->timing & PLK_TIME_PARTIALS) {
    hipEventRecord(ev.b, h->stream);
    h->events.push_back(ev);
  }
  dr_sum_kernel<<<(unsigned)br.size(), 256, 0, h->stream>>>(h->d_drb, a.blk1, a.blk2, n_blk, h->dr_out, h->dr_out + nn);
  HIPCHK(h, hipGetLastError());
  std::vector<double> out(2 * (size_t)nn);
  HIPCHK(h, hipMemcpyAsync(out.data(), h->dr_out, out.size() * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  if (d1) std::copy(out.begin(), out.begin() + nn, d1);
  if (d2) std::copy(out.begin() + nn, out.end(), d2);
  return PLK_OK;
}

}  // namespace

extern "C" {

int plk_update_partials(plk_handle h, const plk_op* ops, int n_ops) {
  env_refresh();
  if (h && !h->shards.empty()) return multi_each(h, [&](plk_handle x) { return plk_update_partials(x, ops, n_ops); });
  if (!h || n_ops < 0 || (n_ops > 0 && !ops)) return fail(h, PLK_ERR_ARG, "bad op list");
  if (n_ops == 0) return PLK_OK;
  hipSetDevice(h->device);
  // the last call's list again (an optimiser's evaluations): its checks hold still -- every
  // condition validate_ops tests is monotonic (matrices, tip codes) except the partial an
  // ACCUMULATE op extends, so only such lists are checked again
  const bool repeat = h->trav_ops.size() == (size_t)n_ops &&
                      std::memcmp(h->trav_ops.data(), ops, n_ops * sizeof(plk_op)) == 0;
  bool accumulate = false;
  if (repeat)
    for (int i = 0; i < n_ops && !accumulate; ++i) accumulate = (ops[i].flags & PLK_OP_ACCUMULATE) != 0;
  if (!repeat || accumulate) {
    int rc = validate_ops(h, ops, n_ops);
    if (rc) return rc;
  }
  // merge the op list into the tree (skipped when it repeats the last call's list)
  if (!repeat) {
    h->trav_ops.assign(ops, ops + n_ops);
    for (int i = 0; i < n_ops; ++i) {
      std::vector<int>& k = h->topo_kids[ops[i].parent];
      if (!(ops[i].flags & PLK_OP_ACCUMULATE)) k.clear();
      k.insert(k.end(), ops[i].child, ops[i].child + ops[i].n_children);
    }
  }
  if (h->flags & PLK_FLAG_SUBTREE_PATTERNS) return update_compressed(h, ops, n_ops);
  if (tree4_supported(h) && fusable(ops, n_ops)) return update_tree4(h, ops, n_ops);
  return update_levelwise(h, ops, n_ops);
}

int plk_get_partials(plk_handle h, int node, double* out) {
  env_refresh();
  if (h && !h->shards.empty()) return multi_slices(h, [&](plk_handle x, int64_t a) { return plk_get_partials(x, node, out ? out + a * h->C * h->S : nullptr); });
  if (!h || !out || node < h->n_tips || node >= h->n_nodes) return fail(h, PLK_ERR_ARG, "bad internal node %d", node);
  hipSetDevice(h->device);
  if (!h->materialized[node - h->n_tips]) {
    // lnL-only traversal kept this partial in registers: re-run the last traversal
    // materialising every node (same arithmetic, so the values are identical).
    if (h->prog_ops.empty()) return fail(h, PLK_ERR_STATE, "node %d has no partial yet", node);
    const unsigned saved = h->flags;
    const std::vector<plk_op> ops = h->prog_ops;
    h->flags &= ~(unsigned)PLK_FLAG_LNL_ONLY;
    const int rc = update_tree4(h, ops.data(), (int)ops.size());
    h->flags = saved;
    if (rc) return rc;
    if (!h->materialized[node - h->n_tips]) return fail(h, PLK_ERR_STATE, "node %d has no partial", node);
  }
  HIPCHK(h, hipStreamSynchronize(h->stream));
  std::vector<double> buf(h->slot_stride);
  HIPCHK(h, hipMemcpy(buf.data(), h->partials + (size_t)(node - h->n_tips) * h->slot_stride,
                      buf.size() * sizeof(double), hipMemcpyDeviceToHost));
  const int CS = h->C * h->S;
  // compressed node: its slot holds one entry per distinct subtree pattern
  const std::vector<int32_t>* ids = nullptr;
  if ((h->flags & PLK_FLAG_SUBTREE_PATTERNS) && h->cmp_valid && !h->slots_expanded &&
      !h->cmp_ids[node - h->n_tips].empty())
    ids = &h->cmp_ids[node - h->n_tips];
  for (int64_t p = 0; p < h->n_patterns; ++p) {
    const int64_t j = ids ? (*ids)[(size_t)p] : p;
    const int64_t tile = j / kTile, q = j % kTile;
    for (int cs = 0; cs < CS; ++cs) out[p * CS + cs] = buf[(tile * CS + cs) * kTile + q];
  }
  return PLK_OK;
}

static int launch_root(plk_handle h, int root);
static int multi_root_loglik(plk_handle h, int root, double* lnl, double* site_lnl, double* block_sums);

}  // extern "C"

namespace {

// A communicator run's global lnL is every rank's block sums in rank order (ranks hold
// consecutive pattern ranges), each rank's in block order -- the same sequence of adds as one
// process over all patterns.  That sequence is one dependent chain of adds, which the host
// runs faster than one GPU thread (~4 vs ~10 cycles per add at a few GHz: 1 960 adds at eight
// ranks of 1 M patterns); this kernel only moves the gathered block sums, and this rank's
// own, into mapped host memory, every thread a share.
__global__ void comm_copy_kernel(const double* __restrict__ all, int64_t n_all, const double* __restrict__ local,
                                 int64_t n_local, double* __restrict__ all_out, double* __restrict__ local_out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_all + n_local;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (i < n_all)
      all_out[i] = all[i];
    else
      local_out[i - n_all] = local[i - n_all];
  }
}

// block sums land in mapped host memory, or in the all-gather's send buffer under a communicator
double* block_target(plk_handle h) { return h->comm ? h->d_blk_local : h->block_sums; }

// The classes' root terms of a one-class-per-workgroup traversal -> site lnL and block sums
// (cls_blocks_kernel) into h->fused_cls_blocks
// (site: also the per-pattern lnL -- an evaluation that returns only the lnL skips those stores)
void launch_cls_blocks(plk_handle h, int guard, int32_t* uflow, bool site) {
  const int n_waves = (int)((h->n_patterns + 63) / 64);
  const dim3 g((unsigned)h->n_blocks), b(1024);
  double* sl = site ? h->site_lnl : nullptr;
  h->cls_site_written = site;
  switch (h->C) {
    case 1: cls_blocks_kernel<1><<<g, b, 0, h->stream>>>(h->d_cls, h->n_pad, h->weights, sl,
                                                        h->fused_cls_blocks, h->n_patterns, n_waves, guard, uflow); break;
    case 2: cls_blocks_kernel<2><<<g, b, 0, h->stream>>>(h->d_cls, h->n_pad, h->weights, sl,
                                                        h->fused_cls_blocks, h->n_patterns, n_waves, guard, uflow); break;
    default: cls_blocks_kernel<4><<<g, b, 0, h->stream>>>(h->d_cls, h->n_pad, h->weights, sl,
                                                         h->fused_cls_blocks, h->n_patterns, n_waves, guard, uflow);
  }
}

// The fixed-order 4096-pattern block sums of the wave sums; under a communicator also the
// underflow flag into this rank's exchange record (plk_exchange.hpp layout).
int launch_block_sums(plk_handle h) {
  const int n_waves = (int)((h->n_patterns + 63) / 64);
  wave_sums_to_blocks<<<(h->n_blocks + 3) / 4, 256, 0, h->stream>>>(
      h->wave_sums, block_target(h), n_waves, h->n_blocks, h->comm ? h->d_uflow : nullptr,
      h->comm ? h->d_blk_local + h->comm_stride - 1 : nullptr);
  HIPCHK(h, hipGetLastError());
  return PLK_OK;
}

// Enqueue the root reduction of `root` (fused traversals already did it), the fixed-order
// 4096-pattern block sums, the RCCL exchange under a communicator, and the per-pattern lnL
// copy; root_finish waits and sums.  Split so that a multi-device handle can have every
// device's reduction in flight before it waits for the first.
int root_launch(plk_handle h, int root, double* site_lnl) {
  if (root < h->n_tips || root >= h->n_nodes) return fail(h, PLK_ERR_ARG, "bad root node %d", root);
  if (!h->pi_set || !h->rates_set) return fail(h, PLK_ERR_STATE, "root frequencies / category rates not set");
  hipSetDevice(h->device);
  if (h->fused_lnl_valid && h->fused_lnl_root == root) {
    // the fused traversal already reduced the root: only the block sums remain (with one class
    // per workgroup they are formed too -- again if the communicator changed where they go)
    if (h->fused_cls_blocks && h->fused_cls_blocks == block_target(h) && (h->cls_site_written || !site_lnl)) {
      if (h->comm) {
        flag_slot_kernel<<<1, 1, 0, h->stream>>>(h->d_uflow, h->d_blk_local + h->comm_stride - 1);
        HIPCHK(h, hipGetLastError());
      }
    } else if (h->fused_cls_blocks) {
      // again: block sums to the communicator's buffer, or the per-pattern lnL asked for
      h->fused_cls_blocks = block_target(h);
      launch_cls_blocks(h, (h->flags & PLK_FLAG_NONNEG_GUARD) ? 1 : 0,
                        (h->flags & PLK_FLAG_SCALING) ? nullptr : h->d_uflow, site_lnl != nullptr);
      HIPCHK(h, hipGetLastError());
      if (h->comm) flag_slot_kernel<<<1, 1, 0, h->stream>>>(h->d_uflow, h->d_blk_local + h->comm_stride - 1);
    } else {
      int rc = launch_block_sums(h);
      if (rc) return rc;
    }
  } else {
    if (!h->materialized[root - h->n_tips]) return fail(h, PLK_ERR_STATE, "root %d has no partial", root);
    int rc = launch_root(h, root);
    if (rc) return rc;
    // the wave sums and block sums of the fused root reduction are overwritten
    h->fused_lnl_valid = false;
    }
  if (h->comm) {
    // the one cross-GPU exchange of an evaluation: a fixed-size all-gather of block sums
    if (ncclAllGather(h->d_blk_local, h->d_blk_all, (size_t)h->comm_stride, ncclFloat64, h->comm, h->stream) !=
        ncclSuccess)
      return fail(h, PLK_ERR_DEVICE, "ncclAllGather of the block sums failed");
    const int64_t n_all = (int64_t)h->comm_ranks * h->comm_stride;
    comm_copy_kernel<<<(unsigned)((n_all + h->n_blocks + 255) / 256), 256, 0, h->stream>>>(
        h->d_blk_all, n_all, h->d_blk_local, h->n_blocks, h->d_blk_all_map, h->block_sums);
    HIPCHK(h, hipGetLastError());
  }
  if (site_lnl)
    HIPCHK(h, hipMemcpyAsync(site_lnl, h->site_lnl, (size_t)h->n_patterns * sizeof(double), hipMemcpyDeviceToHost,
                             h->stream));
  return PLK_OK;
}

// PLK_DEBUG_CLOCK: one record per stamped traversal, from its workgroups' stamps --
// [0] shader clock in MHz over all workgroups (sum of clock ticks / sum of 100 MHz ticks),
// [1] / [2] the slowest / fastest workgroup's, [3] first start to last end in us, [4] workgroups
void clock_summary(plk_handle h) {
  if (!h->clk_n) return;
  double sc = 0.0, sw = 0.0, lo = 1e30, hi = 0.0;
  unsigned long long w0 = ~0ull, w1 = 0;
  for (size_t i = 0; i < h->clk_n; ++i) {
    const volatile unsigned long long* q = h->h_clk + 4 * i;
    const double dc = (double)(q[2] - q[0]), dw = (double)(q[3] - q[1]);
    if (dw <= 0.0) continue;
    sc += dc;
    sw += dw;
    lo = std::min(lo, 100.0 * dc / dw);
    hi = std::max(hi, 100.0 * dc / dw);
    w0 = std::min<unsigned long long>(w0, (unsigned long long)q[1]);
    w1 = std::max<unsigned long long>(w1, (unsigned long long)q[3]);
  }
  const double rec[5] = {sw > 0 ? 100.0 * sc / sw : 0.0, lo, hi, w1 > w0 ? (double)(w1 - w0) / 100.0 : 0.0,
                         (double)h->clk_n};
  h->clk_rec.insert(h->clk_rec.end(), rec, rec + 5);
  h->clk_n = 0;
}

int root_finish(plk_handle h, double* lnl, double* block_sums, bool wait = true) {
  hipSetDevice(h->device);
  if (wait)
    if (int rc = stream_wait(h)) return rc;
  clock_summary(h);  // (the stream has drained: root_finish reads the block sums below)
  double s = 0.0;
  if (h->comm) {
    // rank order, block order (comm_copy_kernel moved the records), and every rank's flag
    s = xchg::reduce(h->h_blk_all, h->comm_counts.data(), h->comm_ranks, h->comm_stride, &h->comm_uflow);
  } else {
    for (int b = 0; b < h->n_blocks; ++b) s += h->h_blocks[b];  // fixed order: block 0, 1, 2, ...
  }
  if (lnl) *lnl = s;
  if (block_sums) std::memcpy(block_sums, h->h_blocks, (size_t)h->n_blocks * sizeof(double));
  return PLK_OK;
}

// Under a communicator: v[0..n) (this rank's derivative sums) becomes the sum over all ranks
// in rank order -- one ncclAllGather of n doubles per rank on the handle's stream, then the
// same chain of adds on every rank, so all ranks return the same doubles (an all-reduce's
// order depends on the ring).  Without a communicator v is left as it is.
int comm_sum_values(plk_handle h, double* v, size_t n) {
  if (!h->comm || n == 0) return PLK_OK;
  hipSetDevice(h->device);
  const size_t R = (size_t)h->comm_ranks;
  int rc = ensure_cap(h, (void**)&h->d_xch, &h->d_xch_cap, n * sizeof(double));
  if (!rc) rc = ensure_cap(h, (void**)&h->d_xch_all, &h->d_xch_all_cap, R * n * sizeof(double));
  if (rc) return rc;
  HIPCHK(h, hipMemcpyAsync(h->d_xch, v, n * sizeof(double), hipMemcpyHostToDevice, h->stream));
  if (ncclAllGather(h->d_xch, h->d_xch_all, n, ncclFloat64, h->comm, h->stream) != ncclSuccess)
    return fail(h, PLK_ERR_DEVICE, "ncclAllGather of the derivative sums failed");
  std::vector<double> all(R * n);
  HIPCHK(h, hipMemcpyAsync(all.data(), h->d_xch_all, all.size() * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  xchg::rank_sums(all.data(), (int)R, n, v);
  return PLK_OK;
}

}  // namespace

extern "C" {

int root_launch_c(plk_handle h, int root, double* site_lnl) { return root_launch(h, root, site_lnl); }
int root_finish_c(plk_handle h, double* lnl, double* block_sums) { return root_finish(h, lnl, block_sums); }

static int multi_root_loglik(plk_handle h, int root, double* lnl, double* site_lnl, double* block_sums) {
  return multi_root_loglik_impl(h, root, lnl, site_lnl, block_sums);
}

int plk_create_multi(const int* devices, int n_devices, int n_states, int n_classes, int64_t n_patterns, int n_tips,
                     int n_internal, int n_models, unsigned flags, plk_handle* out) {
  env_refresh();
  if (!out || !devices || n_devices < 1) return fail(nullptr, PLK_ERR_ARG, "bad device list");
  *out = nullptr;
  if (n_patterns < 1) return fail(nullptr, PLK_ERR_ARG, "bad pattern count");
  plk_handle h = new plk_handle_s();
  h->S = n_states;
  h->C = n_classes;
  h->n_tips = n_tips;
  h->n_internal = n_internal;
  h->n_nodes = n_tips + n_internal;
  h->n_models = n_models;
  h->flags = flags;
  h->n_patterns = n_patterns;
  h->n_blocks = (int)((n_patterns + kRootBlock - 1) / kRootBlock);
  h->device = devices[0];
  // contiguous block-aligned ranges (the last takes the remainder); fewer shards than
  // devices when there are fewer blocks than devices
  const int64_t nb = h->n_blocks;
  const int nd = (int)std::min<int64_t>(n_devices, nb);
  const int64_t per = nb / nd, extra = nb % nd;
  int64_t b = 0;
  for (int i = 0; i < nd; ++i) {
    const int64_t cnt = per + (i < extra ? 1 : 0);
    const int64_t a = b * kRootBlock;
    b += cnt;
    const int64_t e = std::min<int64_t>(b * kRootBlock, n_patterns);
    plk_handle s = nullptr;
    const int rc = plk_create(devices[i], n_states, n_classes, e - a, n_tips, n_internal, n_models, flags, &s);
    if (rc) {
      const std::string msg = g_last_error;
      plk_destroy(h);
      return fail(nullptr, rc, "plk_create_multi: shard %d on device %d: %s", i, devices[i], msg.c_str());
    }
    h->shards.push_back(s);
    h->shard_start.push_back(a);
  }
  h->shard_start.push_back(n_patterns);
  *out = h;
  return PLK_OK;
}

int plk_exchange_stride(const int64_t* counts, int n_ranks, int64_t* stride) {
  if (!counts || !stride || n_ranks < 1) return fail(nullptr, PLK_ERR_ARG, "bad exchange layout arguments");
  const int64_t s = xchg::stride(counts, n_ranks);
  if (s < 1) return fail(nullptr, PLK_ERR_ARG, "negative block count");
  *stride = s;
  return PLK_OK;
}

int plk_exchange_pack(const double* block_sums, int64_t n_blocks, int uflow, int64_t stride, double* record) {
  if (!record || n_blocks < 0 || (n_blocks > 0 && !block_sums) || stride < n_blocks + 1)
    return fail(nullptr, PLK_ERR_ARG, "bad exchange record (%lld blocks, stride %lld)", (long long)n_blocks,
                (long long)stride);
  xchg::pack(block_sums, n_blocks, uflow, stride, record);
  return PLK_OK;
}

int plk_exchange_reduce(const double* gathered, const int64_t* counts, int n_ranks, int64_t stride, double* lnl,
                        int* uflow) {
  if (!gathered || !counts || !lnl || n_ranks < 1) return fail(nullptr, PLK_ERR_ARG, "bad exchange reduce arguments");
  for (int r = 0; r < n_ranks; ++r)
    if (counts[r] < 0 || counts[r] > stride - 1)
      return fail(nullptr, PLK_ERR_ARG, "rank %d: %lld blocks in a record of stride %lld", r, (long long)counts[r],
                  (long long)stride);
  *lnl = xchg::reduce(gathered, counts, n_ranks, stride, uflow);
  return PLK_OK;
}

int plk_exchange_rank_sums(const double* gathered, int n_ranks, int64_t n, double* v) {
  if (!gathered || !v || n_ranks < 1 || n < 0) return fail(nullptr, PLK_ERR_ARG, "bad rank-sum arguments");
  xchg::rank_sums(gathered, n_ranks, (size_t)n, v);
  return PLK_OK;
}

int plk_clock_records(plk_handle h, double* out, int cap, int* n) {
  if (!h || !n || cap < 0 || (cap > 0 && !out)) return fail(h, PLK_ERR_ARG, "bad clock-record arguments");
  const int have = (int)(h->clk_rec.size() / 5);
  *n = have;
  if (out) std::memcpy(out, h->clk_rec.data(), (size_t)std::min(cap, have) * 5 * sizeof(double));
  if (cap >= have) h->clk_rec.clear();
  return PLK_OK;
}

int plk_root_underflow(plk_handle h, int* flag) {
  if (!h || !flag) return fail(h, PLK_ERR_ARG, "null argument");
  if (h->flags & PLK_FLAG_SCALING) return fail(h, PLK_ERR_STATE, "a scaled handle's reduction has no underflow flag");
  int f = 0;
  if (!h->shards.empty()) {
    for (plk_handle x : h->shards) f |= *(volatile int32_t*)x->h_uflow;
  } else if (h->comm) {
    f = h->comm_uflow;  // every rank's flag, carried in the block-sum all-gather
  } else {
    f = *(volatile int32_t*)h->h_uflow;
  }
  *flag = f ? 1 : 0;
  return PLK_OK;
}

int plk_shard_count(plk_handle h, int* n_shards) {
  if (!h || !n_shards) return fail(h, PLK_ERR_ARG, "null argument");
  *n_shards = h->shards.empty() ? 1 : (int)h->shards.size();
  return PLK_OK;
}

int plk_root_loglik(plk_handle h, int root, double* lnl, double* site_lnl, double* block_sums) {
  env_refresh();
  if (!h) return fail(h, PLK_ERR_ARG, "null handle");
  if (!h->shards.empty()) return multi_root_loglik(h, root, lnl, site_lnl, block_sums);
  int rc = root_launch(h, root, site_lnl);
  if (rc) return rc;
  return root_finish(h, lnl, block_sums);
}

static int launch_root(plk_handle h, int root) {
  RootArgs a;
  a.partials = h->partials + (size_t)(root - h->n_tips) * h->slot_stride;
  a.scale = h->scale ? h->scale + (size_t)(root - h->n_tips) * h->n_pad : nullptr;
  a.weights = h->weights;
  a.pi = h->pi;
  a.probs = h->probs;
  a.site_lnl = h->site_lnl;
  a.wave_sums = h->wave_sums;
  a.n_patterns = h->n_patterns;
  a.S = h->S;
  a.C = h->C;
  a.guard = (h->flags & PLK_FLAG_NONNEG_GUARD) ? 1 : 0;
  a.uflow = uflow_arm(h);
  EventPair ev;
  if (h->timing & PLK_TIME_ROOT) {
    ev = get_events(h, 2);
    hipEventRecord(ev.a, h->stream);
  }
  root_kernel<<<(unsigned)(h->n_pad / 64), 64, 0, h->stream>>>(a);
  HIPCHK(h, hipGetLastError());
  if (int rc = launch_block_sums(h)) return rc;
  if (h->timing & PLK_TIME_ROOT) {
    hipEventRecord(ev.b, h->stream);
    h->events.push_back(ev);
  }
  return PLK_OK;
}

static int branch_derivatives_local(plk_handle h, int branch, double* d1, double* d2);

int plk_branch_derivatives(plk_handle h, int branch, double* d1, double* d2) {
  env_refresh();
  if (h && !h->shards.empty()) return multi_branch_derivatives(h, branch, d1, d2);
  if (!h) return fail(h, PLK_ERR_ARG, "null handle");
  double v[2] = {0.0, 0.0};
  int rc = branch_derivatives_local(h, branch, &v[0], &v[1]);
  if (!rc) rc = comm_sum_values(h, v, 2);  // global under a communicator
  if (rc) return rc;
  if (d1) *d1 = v[0];
  if (d2) *d2 = v[1];
  return PLK_OK;
}

static int branch_derivatives_local(plk_handle h, int branch, double* d1, double* d2) {
  if (!h || branch < 0 || branch >= h->n_nodes) return fail(h, PLK_ERR_ARG, "bad branch %d", branch);
  if (h->trav_ops.empty()) return fail(h, PLK_ERR_STATE, "no traversal yet (plk_update_partials)");
  if (h->S != 4 || !(h->C == 1 || h->C == 2 || h->C == 4))
    return path_derivatives(h, branch, d1, d2);
  if (h->deriv_valid.empty() || !h->deriv_valid[branch])
    return fail(h, PLK_ERR_STATE, "dP/d2P of branch %d not computed (PLK_DERIV_DP | PLK_DERIV_D2P)", branch);
  if (!h->pi_set || !h->rates_set) return fail(h, PLK_ERR_STATE, "root frequencies / category rates not set");
  hipSetDevice(h->device);
  const int nt = h->n_tips;
  // tree of the last traversal: sons per node (ops merged), parent map
  std::vector<std::vector<int> > kids(h->n_nodes);
  std::vector<int> parent(h->n_nodes, -1);
  // the merged tree of every traversal so far (an incremental call lists only the
  // ancestors of the changed branches)
  for (int n = 0; n < h->n_nodes; ++n)
    for (int c : h->topo_kids[n]) {
      kids[n].push_back(c);
      parent[c] = n;
    }
  if (parent[branch] < 0) return fail(h, PLK_ERR_ARG, "branch %d is not below any node of the last traversal", branch);
  // every partial read along the path must be in HBM at full length: re-materialise if
  // needed (a compressed traversal's slots hold distinct subtree patterns: the derivative
  // re-runs the traversal uncompressed once, until the next compressed traversal)
  bool need = (h->flags & PLK_FLAG_SUBTREE_PATTERNS) && !h->slots_expanded;
  for (int n = parent[branch]; n >= 0; n = parent[n])
    for (int c : kids[n])
      if (c >= nt && !h->materialized[c - nt]) need = true;
  if (need) {
    int rc = materialize_last_traversal(h);
    if (rc) return rc;
  }
  // path program: father of the branch first, then every ancestor up to the root
  std::vector<DInstr> prog;
  int path = branch;
  for (int n = parent[branch]; n >= 0; path = n, n = parent[n]) {
    for (int c : kids[n]) {
      if (c == path) {
        if (path == branch)
          prog.push_back({D_PATH, c < nt ? 1 : 0, c < nt ? c : c - nt, c});
        else
          prog.push_back({D_PATH, 0, 0, c});
      } else if (c < nt) {
        prog.push_back({D_TIP, 0, c, c});
      } else {
        prog.push_back({D_LOAD, 0, c - nt, c});
      }
    }
    prog.push_back({D_STEP, 0, 0, 0});
  }
  prog.push_back({D_END, 0, 0, 0});
  int rc = ensure_cap(h, (void**)&h->d_dprog, &h->d_dprog_cap, prog.size() * sizeof(DInstr));
  if (rc) return rc;
  HIPCHK(h, hipMemcpyAsync(h->d_dprog, prog.data(), prog.size() * sizeof(DInstr), hipMemcpyHostToDevice,
                           h->stream));
  if (!h->d1_sums) {
    if ((rc = dalloc(h, (void**)&h->d1_sums, (size_t)(h->n_pad / 64) * sizeof(double)))) return rc;
    if ((rc = dalloc(h, (void**)&h->d2_sums, (size_t)(h->n_pad / 64) * sizeof(double)))) return rc;
  }
  DerivArgs a;
  a.partials = h->partials;
  a.codes = h->codes;
  a.init = h->code_table;
  a.pi = h->pi;
  a.probs = h->probs;
  a.weights = h->weights;
  a.d1_sums = h->d1_sums;
  a.d2_sums = h->d2_sums;
  a.slot_stride = h->slot_stride;
  a.n_pad = h->n_pad;
  a.n_patterns = h->n_patterns;
  a.n_codes = h->n_codes;
  const int guard = (h->flags & PLK_FLAG_NONNEG_GUARD) ? 1 : 0;
  const dim3 grid((unsigned)(h->n_pad / 256));
  switch (h->C) {
    case 1: deriv_kernel<4, 1><<<grid, 256, 0, h->stream>>>(a, h->d_dprog, h->pmats, h->dpmats, h->d2pmats, guard); break;
    case 2: deriv_kernel<4, 2><<<grid, 256, 0, h->stream>>>(a, h->d_dprog, h->pmats, h->dpmats, h->d2pmats, guard); break;
    case 4: deriv_kernel<4, 4><<<grid, 256, 0, h->stream>>>(a, h->d_dprog, h->pmats, h->dpmats, h->d2pmats, guard); break;
  }
  HIPCHK(h, hipGetLastError());
  // fixed-order host sum of the wave sums (same order for any run)
  const int n_waves = (int)((h->n_patterns + 63) / 64);
  std::vector<double> w1(n_waves), w2(n_waves);
  HIPCHK(h, hipMemcpyAsync(w1.data(), h->d1_sums, n_waves * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipMemcpyAsync(w2.data(), h->d2_sums, n_waves * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  double s1 = 0.0, s2 = 0.0;
  for (int i = 0; i < n_waves; ++i) {
    s1 += w1[i];
    s2 += w2[i];
  }
  if (d1) *d1 = s1;
  if (d2) *d2 = s2;
  return PLK_OK;
}

int plk_root_pair_derivatives(plk_handle h, int a, int b, double alpha, double beta, double* d1, double* d2) {
  env_refresh();
  if (h && !h->shards.empty()) {
    std::vector<double> u(h->shards.size()), v(h->shards.size());
    const int rc = multi_run(h, [&](size_t i) { return plk_root_pair_derivatives(h->shards[i], a, b, alpha, beta, &u[i], &v[i]); });
    if (rc) return rc;
    double s1 = 0.0, s2 = 0.0;
    for (size_t i = 0; i < u.size(); ++i) {  // shard order
      s1 += u[i];
      s2 += v[i];
    }
    if (d1) *d1 = s1;
    if (d2) *d2 = s2;
    return PLK_OK;
  }
  if (!h) return fail(h, PLK_ERR_ARG, "null handle");
  double v[2] = {0.0, 0.0};
  int rc = root_pair_derivatives(h, a, b, alpha, beta, &v[0], &v[1]);
  if (!rc) rc = comm_sum_values(h, v, 2);
  if (rc) return rc;
  if (d1) *d1 = v[0];
  if (d2) *d2 = v[1];
  return PLK_OK;
}

int plk_set_timing(plk_handle h, int enable) {
  if (h && !h->shards.empty()) return multi_each(h, [&](plk_handle x) { return plk_set_timing(x, enable); });
  if (!h) return fail(h, PLK_ERR_ARG, "null handle");
  h->timing = (unsigned)enable;
  return PLK_OK;
}

int plk_get_timing(plk_handle h, int64_t* n_launches, double* partials_ms, double* pmat_ms, double* root_ms) {
  if (h && !h->shards.empty()) return multi_forward(h, plk_get_timing(h->shards[0], n_launches, partials_ms, pmat_ms, root_ms));
  if (!h) return fail(h, PLK_ERR_ARG, "null handle");
  hipSetDevice(h->device);
  int rc = collect_events(h);
  if (rc) return rc;
  if (n_launches) *n_launches = h->n_launches;
  if (partials_ms) *partials_ms = h->acc_ms[0];
  if (pmat_ms) *pmat_ms = h->acc_ms[1];
  if (root_ms) *root_ms = h->acc_ms[2];
  return PLK_OK;
}

int plk_reset_timing(plk_handle h) {
  if (h && !h->shards.empty()) {
    h->fan_us.assign(h->fan_us.size(), 0.0);
    h->fan_spread_sum = h->fan_spread_max = 0.0;
    h->fan_n = 0;
    return multi_each(h, [&](plk_handle x) { return plk_reset_timing(x); });
  }
  if (!h) return fail(h, PLK_ERR_ARG, "null handle");
  int rc = collect_events(h);
  if (rc) return rc;
  h->n_launches = h->n_table_launches = 0;
  h->acc_ms[0] = h->acc_ms[1] = h->acc_ms[2] = h->acc_ms[3] = 0.0;
  for (double& x : h->host_us) x = 0.0;
  h->n_evals = 0;
  h->last_eval_end = std::chrono::steady_clock::time_point{};
  return PLK_OK;
}

int plk_get_timing_ex(plk_handle h, plk_timing* out) {
  if (h && !h->shards.empty()) return multi_forward(h, plk_get_timing_ex(h->shards[0], out));
  if (!h || !out) return fail(h, PLK_ERR_ARG, "null argument");
  hipSetDevice(h->device);
  int rc = collect_events(h);
  if (rc) return rc;
  out->partials_launches = h->n_launches;
  out->partials_ms = h->acc_ms[0];
  out->pmat_ms = h->acc_ms[1];
  out->root_ms = h->acc_ms[2];
  out->tables_ms = h->acc_ms[3];
  out->table_launches = h->n_table_launches;
  out->evaluations = h->n_evals;
  for (int i = 0; i < 6; ++i) out->host_us[i] = h->host_us[i];
  return PLK_OK;
}

int plk_traversal_work(plk_handle h, plk_work* out) {
  if (h && !h->shards.empty()) return multi_traversal_work(h, out);
  if (!h || !out) return fail(h, PLK_ERR_ARG, "null argument");
  if (h->kernel_path.empty()) return fail(h, PLK_ERR_STATE, "no traversal yet");
  traversal_work(h, out);
  return PLK_OK;
}

int plk_synchronize(plk_handle h) {
  if (h && !h->shards.empty()) return multi_each(h, [&](plk_handle x) { return plk_synchronize(x); });
  if (!h) return fail(h, PLK_ERR_ARG, "null handle");
  hipSetDevice(h->device);
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return PLK_OK;
}

int plk_evaluate(plk_handle h, int n, const int32_t* branch, const int32_t* model, const double* t,
                 const plk_op* ops, int n_ops, int root, double* lnl, double* block_sums) {
  env_refresh();
  if (h && !h->shards.empty()) return multi_evaluate(h, n, branch, model, t, ops, n_ops, root, lnl, block_sums);
  if (!h) return fail(h, PLK_ERR_ARG, "null handle");
  const clk::time_point t0 = clk::now();
  auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
  h->in_eval = true;
  int rc = plk_update_pmatrices(h, n, branch, model, t, PLK_DERIV_P);
  h->in_eval = false;
  if (rc) return rc;
  const clk::time_point t1 = clk::now();
  rc = plk_update_partials(h, ops, n_ops);
  if (rc) return rc;
  const clk::time_point t2 = clk::now();
  rc = root_launch(h, root, nullptr);
  if (rc) return rc;
  const clk::time_point t3 = clk::now();
  if ((rc = stream_wait(h))) return rc;
  h->req_unrecorded = false;  // the staging's reader is done
  const clk::time_point t4 = clk::now();
  rc = root_finish(h, lnl, block_sums, false);
  if (rc) return rc;
  const clk::time_point t5 = clk::now();
  h->host_us[0] += us(t0, t1);
  h->host_us[1] += us(t1, t2);
  h->host_us[2] += us(t2, t3);
  h->host_us[3] += us(t3, t4);
  h->host_us[4] += us(t4, t5);
  if (h->n_evals > 0) h->host_us[5] += us(h->last_eval_end, t0);
  h->n_evals++;
  h->last_eval_end = t5;
  h->t_launched = t2;
  h->t_waited = t4;
  return PLK_OK;
}

int plk_get_fanout(plk_handle h, int n_shards, double* offsets_us, double* spread_us, int64_t* evaluations) {
  if (!h) return fail(h, PLK_ERR_ARG, "null handle");
  const int ns = h->shards.empty() ? 1 : (int)h->shards.size();
  if (n_shards != ns) return fail(h, PLK_ERR_ARG, "handle has %d shard(s), not %d", ns, n_shards);
  const double k = h->fan_n > 0 ? 1.0 / (double)h->fan_n : 0.0;
  for (int i = 0; i < 3 * ns; ++i)
    if (offsets_us) offsets_us[i] = (size_t)i < h->fan_us.size() ? h->fan_us[i] * k : 0.0;
  if (spread_us) {
    spread_us[0] = h->fan_spread_sum * k;
    spread_us[1] = h->fan_spread_max;
  }
  if (evaluations) *evaluations = h->fan_n;
  return PLK_OK;
}

int plk_all_branch_derivatives(plk_handle h, double* d1, double* d2) {
  env_refresh();
  if (h && !h->shards.empty()) return multi_all_branch_derivatives(h, d1, d2);
  if (!h) return fail(h, PLK_ERR_ARG, "null handle");
  if (!h->comm) return dr_derivatives(h, d1, d2);
  const size_t n = (size_t)h->n_nodes;
  std::vector<double> v(2 * n, 0.0);
  int rc = dr_derivatives(h, v.data(), v.data() + n);
  if (!rc) rc = comm_sum_values(h, v.data(), 2 * n);
  if (rc) return rc;
  if (d1) std::memcpy(d1, v.data(), n * sizeof(double));
  if (d2) std::memcpy(d2, v.data() + n, n * sizeof(double));
  return PLK_OK;
}

const char* plk_kernel_path(plk_handle h) {
  if (h && !h->shards.empty()) return plk_kernel_path(h->shards[0]);
  return h ? h->kernel_path.c_str() : "";
}

int plk_compressed_work(plk_handle h, int64_t* updates) {
  if (h && !h->shards.empty()) return multi_compressed_work(h, updates);
  if (!h || !updates) return fail(h, PLK_ERR_ARG, "null argument");
  if (!(h->flags & PLK_FLAG_SUBTREE_PATTERNS) || !h->cmp_valid)
    return fail(h, PLK_ERR_STATE, "no compressed traversal yet");
  *updates = h->cmp_work;
  return PLK_OK;
}

}  // extern "C"
