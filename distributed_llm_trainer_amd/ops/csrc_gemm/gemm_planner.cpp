// Native GEMM planner: hipBLASLt with per-shape autotuned algorithm selection.
//
// The engine's projection GEMMs are plain library GEMMs (bf16 x bf16 -> bf16, and
// bf16 x bf16 -> fp32 accumulated into the fp32 main-grad buffer for weight
// gradients).  Measured on MI355X (tools/cpp/hipblaslt_sweep.cpp, random data), the
// solution the framework's default path picks for the weight-gradient GEMMs
// (dW[N,K] += dY^T X with K_red = B*S = 8192) runs at 180-620 TF/s, while the best
// hipBLASLt solution for the same problem runs 1.3-2x faster.  This planner:
//   * maps row-major PyTorch tensors onto column-major hipBLASLt descriptors,
//   * keys a plan cache on (opA, opB, m, n, k, lds, dtypes, beta != 0),
//   * on the first call of a key, times up to DLT_GEMM_CANDIDATES heuristic
//     solutions on the caller's stream and keeps the fastest (a key first seen
//     inside a HIP-graph capture takes heuristic #0 without timing),
//   * owns one hipBLASLt handle and one device workspace per stream
//     (DLT_GEMM_WORKSPACE_MB, default 64), so GEMMs on the compute and side streams
//     can run concurrently (see StreamCtx),
//   * records the chosen kernel's name for the plan report,
//   * accepts pinned picks (dlt_gemm_pin: key -> hipBLASLt solution index, from
//     hipblaslt_ext::getIndexFromAlgo) so a run replays another run's choices without
//     timing (ops/gemm.py DLT_GEMM_PLAN, the shipped configs/gemm_plan_mi355x.json);
//     a pin this hipBLASLt build does not support for the problem is ignored,
//   * DLT_GEMM_TUNE=exhaustive times EVERY supported solution (getAllAlgos), not just
//     the heuristic's first candidates: 2-15 % faster picks on the model's shapes
//     (profiles/r2_gemm_exhaustive.md), minutes of tuning -> an offline step.
// C ABI, loaded by ctypes from ops/gemm.py.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <hipblaslt/hipblaslt-ext.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#define DLT_API extern "C" __attribute__((visibility("default")))

namespace {

struct Key {
  int ta, tb, m, n, k, lda, ldb, ldc, dta, dtb, dtc, accumulate;
  int batch = 1;  // strided-batched (split-K wgrad): element strides of A, B, C
  long long sa = 0, sb = 0, sc = 0;
  bool operator<(const Key& o) const {
    return std::tie(ta, tb, m, n, k, lda, ldb, ldc, dta, dtb, dtc, accumulate, batch, sa, sb, sc) <
           std::tie(o.ta, o.tb, o.m, o.n, o.k, o.lda, o.ldb, o.ldc, o.dta, o.dtb, o.dtc, o.accumulate, o.batch, o.sa,
                    o.sb, o.sc);
  }
};

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo;
  size_t ws = 0;
  float us = -1.f;
  int chosen = 0, candidates = 0;
  int sol = -1;  // hipBLASLt solution index (stable within one hipBLASLt build)
  std::string kernel;
};

// Per-stream execution context: a hipBLASLt handle of its own plus a workspace.  A
// handle is not safe for GEMMs in flight concurrently on two streams: the gfx950
// kernels are stream-K "UserArgs" kernels and sharing one handle between the compute
// and side streams deadlocked the GPU (100 % busy, spinning workgroups) within a few
// pipelined training steps; one handle per stream does not.
struct StreamCtx {
  hipblasLtHandle_t h = nullptr;
  void* ws = nullptr;
};

struct Planner {
  hipblasLtHandle_t h = nullptr;    // heuristics / autotune / kernel-name queries
  std::map<hipStream_t, StreamCtx> ctx;  // one handle + workspace per stream
  size_t wsz = 0;
  std::map<Key, Plan> plans;
  std::mutex mu;
  int max_cand = 24;
  bool tune = true;
  bool verbose = false;
  bool drain = true;  // DLT_GEMM_TUNE_DRAIN=0: time candidates without draining the device first
  bool fail_backup = false;  // test hook: behave as if the accumulator backup could not be allocated
  std::map<Key, int> pins;   // key -> hipBLASLt solution index (replayed plan)
  bool exhaustive = false;   // DLT_GEMM_TUNE=exhaustive: time every supported solution
  int pin_misses = 0;        // pinned solutions this build rejected
};

Planner* g = nullptr;

hipDataType dt_of(int code) { return code == 0 ? HIP_R_32F : (code == 1 ? HIP_R_16BF : HIP_R_16F); }

int init() {
  if (g) return 0;
  Planner* p = new Planner();
  if (hipblasLtCreate(&p->h) != HIPBLAS_STATUS_SUCCESS) return -10;
  const char* e = getenv("DLT_GEMM_WORKSPACE_MB");
  p->wsz = (size_t)(e ? atoi(e) : 64) << 20;
  e = getenv("DLT_GEMM_CANDIDATES");
  if (e) p->max_cand = atoi(e);
  e = getenv("DLT_GEMM_TUNE");
  if (e && strcmp(e, "exhaustive") == 0) p->exhaustive = true;
  else if (e && atoi(e) == 0) p->tune = false;
  e = getenv("DLT_GEMM_VERBOSE");
  p->verbose = e && atoi(e) != 0;
  e = getenv("DLT_GEMM_TUNE_DRAIN");
  if (e && atoi(e) == 0) p->drain = false;
  g = p;
  return 0;
}

// caller holds g->mu
const StreamCtx* stream_ctx(hipStream_t s) {
  auto it = g->ctx.find(s);
  if (it != g->ctx.end()) return &it->second;
  StreamCtx c;
  if (hipblasLtCreate(&c.h) != HIPBLAS_STATUS_SUCCESS) return nullptr;
  if (hipMalloc(&c.ws, g->wsz) != hipSuccess) return nullptr;
  return &g->ctx.emplace(s, c).first->second;
}

bool capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) != hipSuccess) return false;
  return st != hipStreamCaptureStatusNone;
}

int build_plan(const Key& k, Plan& p, const void* A, const void* B, void* C, hipStream_t s, const StreamCtx* sc) {
  void* ws = sc->ws;
  if (hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return -20;
  hipblasOperation_t ta = k.ta ? HIPBLAS_OP_T : HIPBLAS_OP_N, tb = k.tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
  const int ar = k.ta ? k.k : k.m, ac = k.ta ? k.m : k.k;  // stored (rows, cols) of A in col-major
  const int br = k.tb ? k.n : k.k, bc = k.tb ? k.k : k.n;
  if (hipblasLtMatrixLayoutCreate(&p.la, dt_of(k.dta), ar, ac, k.lda) != HIPBLAS_STATUS_SUCCESS) return -21;
  if (hipblasLtMatrixLayoutCreate(&p.lb, dt_of(k.dtb), br, bc, k.ldb) != HIPBLAS_STATUS_SUCCESS) return -22;
  if (hipblasLtMatrixLayoutCreate(&p.lc, dt_of(k.dtc), k.m, k.n, k.ldc) != HIPBLAS_STATUS_SUCCESS) return -23;
  if (k.batch > 1) {
    const int32_t bc32 = k.batch;
    const int64_t st[3] = {k.sa, k.sb, k.sc};
    hipblasLtMatrixLayout_t ls[3] = {p.la, p.lb, p.lc};
    for (int i = 0; i < 3; ++i) {
      hipblasLtMatrixLayoutSetAttribute(ls[i], HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &bc32, sizeof(bc32));
      hipblasLtMatrixLayoutSetAttribute(ls[i], HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &st[i], sizeof(st[i]));
    }
  }
  hipblasLtMatmulPreference_t pref;
  hipblasLtMatmulPreferenceCreate(&pref);
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &g->wsz, sizeof(g->wsz));
  std::vector<hipblasLtMatmulHeuristicResult_t> res(std::max(1, g->max_cand));
  int n = 0;
  hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(g->h, p.desc, p.la, p.lb, p.lc, p.lc, pref,
                                                       (int)res.size(), res.data(), &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (st != HIPBLAS_STATUS_SUCCESS || n == 0) return -24;
  res.resize(n);
  float alpha = 1.f, beta0 = 0.f;
  p.algo = res[0].algo;
  p.ws = res[0].workspaceSize;
  p.candidates = n;
  auto finish = [&](int chosen) {
    p.chosen = chosen;
    p.sol = hipblaslt_ext::getIndexFromAlgo(p.algo);
    p.kernel = hipblaslt_ext::getKernelNameFromAlgo(g->h, p.algo);
  };
  // pinned solution (a replayed plan): the solution index names a kernel of this
  // hipBLASLt build; it is used only if hipBLASLt confirms it supports this problem
  auto pin = g->pins.find(k);
  if (pin != g->pins.end() && pin->second >= 0) {
    std::vector<int> idx{pin->second};
    std::vector<hipblasLtMatmulHeuristicResult_t> r1;
    size_t need = 0;
    if (hipblaslt_ext::getAlgosFromIndex(g->h, idx, r1) == HIPBLAS_STATUS_SUCCESS && !r1.empty() &&
        hipblaslt_ext::matmulIsAlgoSupported(g->h, p.desc, &alpha, p.la, p.lb, &beta0, p.lc, p.lc, r1[0].algo, need) ==
            HIPBLAS_STATUS_SUCCESS &&
        need <= g->wsz) {
      p.algo = r1[0].algo;
      p.ws = need;
      finish(-1);
      return 0;
    }
    (void)hipGetLastError();
    ++g->pin_misses;  // stale plan entry (other hipBLASLt build): fall through to tuning
  }
  if (!g->tune || capturing(s)) {
    finish(0);
    return 0;
  }
  // candidate list: the heuristic's first max_cand, or (DLT_GEMM_TUNE=exhaustive) every
  // solution of this GEMM type that hipBLASLt accepts for the problem -- thousands, so
  // exhaustive tuning is an offline step whose picks are shipped as a plan file
  // (tools/tune_gemm_plan.py, configs/gemm_plan_mi355x.json).
  std::vector<std::pair<hipblasLtMatmulAlgo_t, size_t>> cands;
  for (auto& r : res)  // the heuristic's candidates always compete (first, in its order)
    if (r.workspaceSize <= g->wsz) cands.emplace_back(r.algo, r.workspaceSize);
  size_t n_all = 0;
  if (g->exhaustive) {
    std::vector<int> seen;
    for (auto& c : cands) seen.push_back(hipblaslt_ext::getIndexFromAlgo(c.first));
    std::vector<hipblasLtMatmulHeuristicResult_t> all;
    hipblaslt_ext::getAllAlgos(g->h, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, ta, tb, dt_of(k.dta), dt_of(k.dtb),
                               dt_of(k.dtc), dt_of(k.dtc), HIPBLAS_COMPUTE_32F, all);
    n_all = all.size();
    for (auto& r : all) {
      size_t need = 0;
      if (std::find(seen.begin(), seen.end(), hipblaslt_ext::getIndexFromAlgo(r.algo)) != seen.end()) continue;
      if (hipblaslt_ext::matmulIsAlgoSupported(g->h, p.desc, &alpha, p.la, p.lb, &beta0, p.lc, p.lc, r.algo, need) ==
              HIPBLAS_STATUS_SUCCESS &&
          need <= g->wsz)
        cands.emplace_back(r.algo, need);
    }
    (void)hipGetLastError();
  }
  if (cands.size() <= 1) {
    finish(0);
    return 0;
  }
  // Autotune on the caller's stream.  Timing needs a host sync; this runs once per
  // shape (warmup step).  beta = 0 while timing so an accumulating GEMM does not
  // disturb C (its real call comes right after with the requested beta).
  // Drain the whole device first: with micro-step pipelining the other HIP stream may
  // still be running compute, and under DDP an RCCL all-reduce kernel may be spinning on
  // CUs waiting for a slower peer; either would bias the timings below towards kernels
  // that do well on fewer CUs.  (No deadlock: every collective this rank waits for was
  // launched by it, and peers launch collectives in the same order.)
  if (g->drain) hipDeviceSynchronize();
  size_t csize = (k.batch > 1 ? (size_t)k.sc * (k.batch - 1) : 0) + (size_t)k.ldc * k.n;
  csize *= (k.dtc == 0 ? 4 : 2);
  void* cbak = nullptr;
  if (k.accumulate) {
    // The candidates are timed IN PLACE with beta = 0, which overwrites C.  Without a
    // backup of the accumulator the real beta = 1 call would add to A*B instead of the
    // old C (a silently corrupted gradient), so no backup => no timing: keep the
    // heuristic's first pick.
    if (g->fail_backup || hipMalloc(&cbak, csize) != hipSuccess) {
      (void)hipGetLastError();  // do not let the failed allocation surface at the next launch check
      finish(0);
      return 0;
    }
    hipMemcpyAsync(cbak, C, csize, hipMemcpyDeviceToDevice, s);
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto time_it = [&](hipblasLtMatmulAlgo_t& algo, int warm, int iters) -> float {
    for (int w = 0; w < warm; ++w)
      if (hipblasLtMatmul(sc->h, p.desc, &alpha, A, p.la, B, p.lb, &beta0, C, p.lc, C, p.lc, &algo, ws, g->wsz, s) !=
          HIPBLAS_STATUS_SUCCESS)
        return -1.f;
    hipEventRecord(e0, s);
    for (int it = 0; it < iters; ++it)
      hipblasLtMatmul(sc->h, p.desc, &alpha, A, p.la, B, p.lb, &beta0, C, p.lc, C, p.lc, &algo, ws, g->wsz, s);
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    return ms * 1000.f / iters;
  };
  std::vector<std::pair<float, int>> t;
  const bool two_pass = cands.size() > 32;  // exhaustive: a short screen, then re-time the best 8
  for (int i = 0; i < (int)cands.size(); ++i) {
    const float us = two_pass ? time_it(cands[i].first, 1, 2) : time_it(cands[i].first, 2, 5);
    if (us > 0) t.emplace_back(us, i);
  }
  (void)hipGetLastError();
  std::sort(t.begin(), t.end());
  if (two_pass && t.size() > 1) {
    const int top = std::min<int>(8, (int)t.size());
    for (int j = 0; j < top; ++j) t[j].first = time_it(cands[t[j].second].first, 1, 10);
    std::sort(t.begin(), t.begin() + top);
  }
  if (cbak) {
    hipMemcpyAsync(C, cbak, csize, hipMemcpyDeviceToDevice, s);
    hipStreamSynchronize(s);
    hipFree(cbak);
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  const int bi = t.empty() ? 0 : t[0].second;
  p.algo = cands[bi].first;
  p.ws = cands[bi].second;
  p.us = t.empty() ? -1.f : t[0].first;
  p.candidates = (int)cands.size();
  finish(bi);
  if (g->verbose)
    fprintf(stderr, "[dlt-gemm] ta=%d tb=%d m=%d n=%d k=%d acc=%d: %zu candidates (of %zu solutions), chose #%d sol %d (%.1f us, %.0f TF/s)\n",
            k.ta, k.tb, k.m, k.n, k.k, k.accumulate, cands.size(), n_all, bi, p.sol, p.us,
            2.0 * k.m * k.n * k.k * k.batch / p.us / 1e6);
  return 0;
}

}  // namespace

// C[m,n] (col-major, ldc) = alpha * op(A) * op(B) + beta * C ; dtype codes: 0 fp32, 1 bf16, 2 fp16
static int gemm_impl(Key key, const void* A, const void* B, void* C, float alpha, float beta, hipStream_t s) {
  if (int rc = init()) return rc;
  Plan* p;
  const StreamCtx* sc;
  {
    std::lock_guard<std::mutex> lk(g->mu);
    sc = stream_ctx(s);
    if (!sc) return -11;
    auto it = g->plans.find(key);
    if (it == g->plans.end()) {
      Plan np;
      int rc = build_plan(key, np, A, B, C, s, sc);
      if (rc) return rc;
      it = g->plans.emplace(key, np).first;
    }
    p = &it->second;
  }
  hipblasStatus_t st = hipblasLtMatmul(sc->h, p->desc, &alpha, A, p->la, B, p->lb, &beta, C, p->lc, C, p->lc,
                                       &p->algo, sc->ws, g->wsz, s);
  return st == HIPBLAS_STATUS_SUCCESS ? 0 : -30 - (int)st;
}

DLT_API int dlt_gemm(int ta, int tb, int m, int n, int k, const void* A, int lda, int dta, const void* B, int ldb,
                     int dtb, void* C, int ldc, int dtc, float alpha, float beta, hipStream_t s) {
  Key key{ta, tb, m, n, k, lda, ldb, ldc, dta, dtb, dtc, beta != 0.f ? 1 : 0};
  return gemm_impl(key, A, B, C, alpha, beta, s);
}

// Strided-batched GEMM: `batch` independent problems, operand i at A + i*sa etc.
// (element strides).  Used for split-K weight gradients: the token dimension is cut
// into `batch` slices whose partial dW land in a [batch, n, ldc] fp32 scratch that is
// then summed into the accumulator -- the skinny 768x768 / 768x2304 wgrads have too
// few output tiles to fill 256 CUs with K = 32768 on one tile per CU.
DLT_API int dlt_gemm_batched(int ta, int tb, int m, int n, int k, const void* A, int lda, int dta, long long sa,
                             const void* B, int ldb, int dtb, long long sb, void* C, int ldc, int dtc, long long sc,
                             int batch, float alpha, float beta, hipStream_t s) {
  if (batch < 1) return -5;
  Key key{ta, tb, m, n, k, lda, ldb, ldc, dta, dtb, dtc, beta != 0.f ? 1 : 0};
  key.batch = batch;
  key.sa = sa;
  key.sb = sb;
  key.sc = sc;
  return gemm_impl(key, A, B, C, alpha, beta, s);
}

DLT_API int dlt_gemm_num_plans() { return g ? (int)g->plans.size() : 0; }
DLT_API int dlt_gemm_pin_misses() { return g ? g->pin_misses : 0; }

// hipBLASLt build identifier (solution indices are only meaningful within one build)
DLT_API int dlt_gemm_lib_version() {
  int v = 0;
  if (int rc = init()) return rc;
  hipblasLtGetVersion(g->h, &v);
  return v;
}

// Test hook: pretend the accumulator backup allocation fails (accumulating keys first
// seen afterwards are not timed).
DLT_API int dlt_gemm_test_fail_backup(int on) {
  if (int rc = init()) return rc;
  std::lock_guard<std::mutex> lk(g->mu);
  g->fail_backup = on != 0;
  return 0;
}

// Pin the hipBLASLt solution index of a key (before the key is first used).
DLT_API int dlt_gemm_pin(int ta, int tb, int m, int n, int k, int lda, int ldb, int ldc, int dta, int dtb, int dtc,
                         int accumulate, int batch, long long sa, long long sb, long long sc, int chosen) {
  if (int rc = init()) return rc;
  Key key{ta, tb, m, n, k, lda, ldb, ldc, dta, dtb, dtc, accumulate ? 1 : 0};
  key.batch = batch;
  key.sa = sa;
  key.sb = sb;
  key.sc = sc;
  std::lock_guard<std::mutex> lk(g->mu);
  g->pins[key] = chosen;
  return 0;
}

// Machine-readable plan table: one line per key,
// "ta tb m n k lda ldb ldc dta dtb dtc acc batch sa sb sc solution" (input of dlt_gemm_pin).
DLT_API int dlt_gemm_dump(char* buf, int len) {
  if (!g || len <= 0) return 0;
  std::string out;
  std::lock_guard<std::mutex> lk(g->mu);
  for (auto& kv : g->plans) {
    const Key& k = kv.first;
    char line[256];
    snprintf(line, sizeof(line), "%d %d %d %d %d %d %d %d %d %d %d %d %d %lld %lld %lld %d\n", k.ta, k.tb, k.m, k.n,
             k.k, k.lda, k.ldb, k.ldc, k.dta, k.dtb, k.dtc, k.accumulate, k.batch, k.sa, k.sb, k.sc,
             kv.second.sol);
    out += line;
  }
  if (out.size() + 1 > (size_t)len) return -1;
  memcpy(buf, out.data(), out.size());
  buf[out.size()] = 0;
  return (int)out.size();
}

// Dump the plan table (shape, chosen candidate, measured us) for profiles/ and logs.
DLT_API int dlt_gemm_report(char* buf, int len) {
  if (!g || len <= 0) return 0;
  std::string out;
  for (auto& kv : g->plans) {
    const Key& k = kv.first;
    const Plan& p = kv.second;
    char line[512];
    snprintf(line, sizeof(line), "ta=%d tb=%d m=%d n=%d k=%d acc=%d dtc=%d cand=%d chosen=%d sol=%d us=%.1f %.80s\n",
             k.ta, k.tb, k.m, k.n, k.k, k.accumulate, k.dtc, p.candidates, p.chosen, p.sol, p.us, p.kernel.c_str());
    out += line;
  }
  int n = (int)std::min<size_t>(out.size(), (size_t)len - 1);
  memcpy(buf, out.data(), n);
  buf[n] = 0;
  return n;
}
