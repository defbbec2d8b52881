"""GEMMs of the fused executor through the native hipBLASLt planner (``_dlt_gemm.so``).

Row-major PyTorch operands are mapped onto column-major BLAS calls (a row-major
[r, c] matrix is a column-major [c, r] matrix with ld = c):

  linear       Y[M,N]  = X[M,K] . W[N,K]^T   ->  Y^T = op_T(W_c) . X_c        (m=N, n=M, k=K)
  linear_dgrad dX[M,K] = dY[M,N] . W[N,K]    ->  dX^T = W_c . dY_c            (m=K, n=M, k=N)
  wgrad_acc    dW[N,K] += dY^T . X           ->  dW^T += X_c . op_T(dY_c)     (m=K, n=N, k=M), fp32 C

Each distinct shape is autotuned once on first use (see ``csrc_gemm/gemm_planner.cpp``).
If the planner library cannot be loaded, the engine uses torch.matmul (also hipBLASLt,
default heuristics) and logs why.

Plans.  Autotuning picks the hipBLASLt solution, the split-K factor of the weight
gradients and the hand-written-vs-library races per process by timing, so the
summation order of a weight gradient (and the last bits of a loss curve) can differ
between runs, or between a run and its resumed continuation.  A plan file pins them:
* ``configs/gemm_plan_mi355x.json`` (shipped) holds the picks of an EXHAUSTIVE offline
  search over every hipBLASLt solution for the headline shapes
  (``tools/tune_gemm_plan.py``, ``DLT_GEMM_TUNE=exhaustive``; 2-15 % faster than the
  best of the heuristic's first 24 candidates, ``profiles/r2_gemm_exhaustive.md``).  It
  is loaded by default; keys it does not cover are tuned as usual, and pins a different
  hipBLASLt build does not support are ignored.
* ``DLT_GEMM_PLAN=path`` replaces it: if the file exists every choice is replayed from
  it (no timing); otherwise the first process to finish a step writes it
  (``save_plan``).  ``DLT_GEMM_PLAN=none``: no plan.  ``DLT_GEMM_PLAN_OUT=path`` keeps
  the shipped plan and writes it, merged with the choices raced in this process, to path.
DDP replicas stay in sync regardless (the all-reduced gradient is identical on every
rank).  For bitwise run-to-run reproducibility without a plan file use
``DLT_GEMM_TUNE=0 DLT_WGRAD_SPLITK=0 DLT_GEMM_TN=0 DLT_GEMM_FUSED=0`` (heuristic #0 everywhere).
"""
from __future__ import annotations

import ctypes
import os
import warnings

import torch

_LIB = None
_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_dlt_gemm.so")
_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def lib():
    global _LIB
    if _LIB is None:
        import torch  # noqa: F401  (torch's HIP runtime + hipBLASLt must be loaded first)
        L = ctypes.CDLL(_PATH)
        c = ctypes
        L.dlt_gemm.argtypes = [c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, c.c_void_p, c.c_int, c.c_int, c.c_void_p,
                               c.c_int, c.c_int, c.c_void_p, c.c_int, c.c_int, c.c_float, c.c_float, c.c_void_p]
        L.dlt_gemm.restype = c.c_int
        L.dlt_gemm_batched.argtypes = [c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, c.c_void_p, c.c_int, c.c_int,
                                       c.c_longlong, c.c_void_p, c.c_int, c.c_int, c.c_longlong, c.c_void_p, c.c_int,
                                       c.c_int, c.c_longlong, c.c_int, c.c_float, c.c_float, c.c_void_p]
        L.dlt_gemm_batched.restype = c.c_int
        L.dlt_gemm_report.argtypes = [c.c_char_p, c.c_int]
        L.dlt_gemm_report.restype = c.c_int
        L.dlt_gemm_dump.argtypes = [c.c_char_p, c.c_int]
        L.dlt_gemm_dump.restype = c.c_int
        L.dlt_gemm_pin.argtypes = [c.c_int] * 13 + [c.c_longlong] * 3 + [c.c_int]
        L.dlt_gemm_pin.restype = c.c_int
        L.dlt_gemm_test_fail_backup.argtypes = [c.c_int]
        L.dlt_gemm_test_fail_backup.restype = c.c_int
        L.dlt_gemm_lib_version.argtypes = []
        L.dlt_gemm_lib_version.restype = c.c_int
        L.dlt_gemm_pin_misses.argtypes = []
        L.dlt_gemm_pin_misses.restype = c.c_int
        _LIB = L
        _load_plan_env()
    return _LIB


# ---------------------------------------------------------------- plan pinning
_PINNED = {"tn": {}, "splitk": {}, "hipblaslt": {}}  # replayed choices (see module docstring)
_PLAN_STATE = {"path": None, "loaded": False, "saved": False}
_INSTANCES = []  # weak references to live HipGemm objects (for save_plan)
_RACES = {}  # process-wide race outcomes, see HipGemm.__init__
SHIPPED_PLAN = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                            "configs", "gemm_plan_mi355x.json")


def _load_plan_env() -> None:
    path = os.environ.get("DLT_GEMM_PLAN")
    if path == "none":
        return
    if path:
        _PLAN_STATE["path"] = path
        if os.path.exists(path):
            load_plan(path)
    elif os.path.exists(SHIPPED_PLAN):
        load_plan(SHIPPED_PLAN, shipped=True)
        # DLT_GEMM_PLAN_OUT=path: start from the shipped plan and write the merged plan
        # (shipped pins + this process's new races) after the first step
        _PLAN_STATE["path"] = os.environ.get("DLT_GEMM_PLAN_OUT") or None


def load_plan(path: str, shipped: bool = False) -> None:
    """Pin every choice recorded in a plan file written by :func:`save_plan`.  The
    hipBLASLt solution pins are skipped when the file was tuned with another hipBLASLt
    build (solution indices are build-specific)."""
    import json
    with open(path) as f:
        plan = json.load(f)
    L = lib()
    ver = int(L.dlt_gemm_lib_version())
    if ver < 0:  # planner could not initialise (no GPU): nothing to pin
        return
    if plan.get("hipblaslt_version", ver) != ver:
        warnings.warn(f"GEMM plan {path} was tuned with hipBLASLt {plan.get('hipblaslt_version')}, this is {ver}: "
                      "its solution pins are ignored")
    else:
        for line in plan.get("hipblaslt", []):
            v = [int(x) for x in line.split()]
            if len(v) != 17:
                raise ValueError(f"bad hipBLASLt plan line {line!r} in {path}")
            rc = L.dlt_gemm_pin(*v)
            if rc != 0:
                raise RuntimeError(f"dlt_gemm_pin failed ({rc})")
            _PINNED["hipblaslt"][tuple(v[:-1])] = line
    # "tn": forward-projection race ("bf16" = the persistent hand-written kernel, "fw4" = the
    # one-tile-per-workgroup 4-wave 256 x 256 one with
    # AGPR accumulators (csrc/gemm_fw4.hip; "fw4:<flags>" with its own launch flags), null =
    # hipBLASLt; the
    # round-2 integer tile configs of the retired gemm_tn kernels read as "library");
    # "fused": "kind:MxNxK" -> fused epilogue picked (older keys without a kind are ignored)
    _PINNED["tn"] = {tuple(int(x) for x in k.split("x")): (c if c in ("bf16", "fw4") or str(c).startswith("fw4:") else None)
                     for k, c in plan.get("tn", {}).items()}
    for k, c in plan.get("fused", {}).items():
        if ":" in k:
            kind, dims = k.split(":", 1)
            # "swiglu4": the 4-wave k_gemm_fw4 with the SwiGLU epilogue, value = its launch flags
            # (an int; false / null = not used); every other kind is a bool
            _PINNED["tn"][(kind, *(int(x) for x in dims.split("x")))] = (
                (int(c) if c is not None and c is not False else None) if kind == "swiglu4" else bool(c))
    _PINNED["splitk"] = {_splitk_key(k): int(c) for k, c in plan.get("splitk", {}).items()}
    if _RACES:
        _RACES["tn"].update(_PINNED["tn"])
        _RACES["splitk"].update(_PINNED["splitk"])
    if not shipped:
        _PLAN_STATE["loaded"] = True


def _splitk_key(text: str):
    """'MxNxK' -> (M, N, K); 'MxNxKxbf16' -> (M, N, K, 'bf16') (the 16-bit-output races,
    'bf16' / 'fp16')."""
    parts = text.split("x")
    return tuple(p if p in ("bf16", "fp16") else int(p) for p in parts)


def export_plan() -> dict:
    """Every choice made so far in this process (hipBLASLt heuristic indices, the
    hand-written GEMM race and the split-K factors of all live HipGemm objects)."""
    buf = ctypes.create_string_buffer(1 << 20)
    n = lib().dlt_gemm_dump(buf, len(buf))
    if n < 0:
        raise RuntimeError("plan table too large")
    tn, sk = dict(_PINNED["tn"]), dict(_PINNED["splitk"])
    for ref in _INSTANCES:
        g = ref()
        if g is not None:
            tn.update(g._choice)
            sk.update(g._splitk)
    # pins loaded from a plan but not exercised by this process are carried over
    hl = dict(_PINNED["hipblaslt"])
    for ln in buf.value[:n].decode().splitlines():
        if ln and int(ln.split()[-1]) >= 0:
            hl[tuple(int(x) for x in ln.split()[:-1])] = ln
    return {"hipblaslt_version": int(lib().dlt_gemm_lib_version()),
            "hipblaslt": [hl[k] for k in sorted(hl)],
            "tn": {"x".join(map(str, k)): c for k, c in tn.items() if len(k) == 3},
            "fused": {f"{k[0]}:" + "x".join(map(str, k[1:])): (c if k[0] == "swiglu4" else bool(c))
                      for k, c in tn.items() if len(k) == 4},
            "splitk": {"x".join(map(str, k)): c for k, c in sk.items()}}


def save_plan(path: str) -> None:
    import json
    tmp = f"{path}.tmp{os.getpid()}"
    with open(tmp, "w") as f:
        json.dump(export_plan(), f, indent=1)
    os.replace(tmp, path)


def maybe_save_plan() -> None:
    """Called by the trainers after a step: with ``DLT_GEMM_PLAN`` set and no plan file
    yet, write this process's choices once (rank 0 of a job, or a single process)."""
    path = _PLAN_STATE["path"]
    if _LIB is None or not path or _PLAN_STATE["loaded"] or _PLAN_STATE["saved"]:
        return
    _PLAN_STATE["saved"] = True
    if int(os.environ.get("RANK", "0")) == 0 and not os.path.exists(path):
        save_plan(path)


def race_report() -> dict:
    """Human-readable hand-written-vs-library decisions made so far in this process."""
    for ref in _INSTANCES:
        g = ref()
        if g is not None:
            return g.report_choices()
    return {}


def available() -> bool:
    if not os.path.exists(_PATH):
        return False
    try:
        lib()
        return True
    except OSError as e:  # pragma: no cover
        warnings.warn(f"GEMM planner unavailable ({e}); using torch.matmul")
        return False


def report() -> str:
    buf = ctypes.create_string_buffer(1 << 16)
    n = lib().dlt_gemm_report(buf, len(buf))
    return buf.value[:n].decode()


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _gemm(ta, tb, m, n, k, A, lda, B, ldb, C, ldc, alpha=1.0, beta=0.0):
    rc = lib().dlt_gemm(ta, tb, m, n, k, ctypes.c_void_p(A.data_ptr()), lda, _DT[A.dtype],
                        ctypes.c_void_p(B.data_ptr()), ldb, _DT[B.dtype], ctypes.c_void_p(C.data_ptr()), ldc,
                        _DT[C.dtype], alpha, beta, _stream())
    if rc != 0:
        raise RuntimeError(f"dlt_gemm failed ({rc}) for ta={ta} tb={tb} m={m} n={n} k={k}")


def _gemm_batched(ta, tb, m, n, k, A, lda, sa, B, ldb, sb, C, ldc, sc, batch, alpha=1.0, beta=0.0):
    rc = lib().dlt_gemm_batched(ta, tb, m, n, k, ctypes.c_void_p(A.data_ptr()), lda, _DT[A.dtype], sa,
                                ctypes.c_void_p(B.data_ptr()), ldb, _DT[B.dtype], sb, ctypes.c_void_p(C.data_ptr()),
                                ldc, _DT[C.dtype], sc, batch, alpha, beta, _stream())
    if rc != 0:
        raise RuntimeError(f"dlt_gemm_batched failed ({rc}) for ta={ta} tb={tb} m={m} n={n} k={k} batch={batch}")


def _rowmajor(t: torch.Tensor) -> int:
    """Leading dimension of a row-major 2-D tensor (must be unit-stride in dim 1)."""
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError("GEMM operand must be 2-D with unit inner stride")
    return t.stride(0)


def _time_of(fn, reps: int = 3, inner: int = 5) -> float:
    """Best-of-``reps`` device time (ms) of ``inner`` back-to-back calls of ``fn``."""
    fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(inner):
            fn()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best


class HipGemm:
    """The engine's GEMM interface: hand-written MFMA kernels (``csrc/gemm_bf16.hip``)
    and the autotuned hipBLASLt planner (one hipBLASLt handle + workspace per stream, so
    GEMMs on the compute and side streams may overlap).

    Forward projections race the hand-written persistent kernel against the planner's
    pick once per shape and keep the faster (``DLT_GEMM_TN=0``: library only).  The two
    fused forms race the same way, each against its unfused equivalent:
      * ``linear_rope``   -- QKV projection with RoPE in the epilogue vs GEMM + ``rope_qk_inplace``
      * ``linear_swiglu`` -- gate/up projection with SwiGLU in the epilogue vs GEMM + ``swiglu_fwd``
    Choices are process-wide (one summation order per shape) and pinned by plan files."""

    stream_safe = True

    SPLITK_CANDIDATES = (2, 4, 8, 16)
    # a hand-written candidate must beat the library by this factor to be picked (the
    # timings are taken in place during the first step and are a few % noisy)
    RACE_MARGIN = 0.97

    def __init__(self):
        import weakref
        lib()  # loads DLT_GEMM_PLAN pins before any choice is made
        # race outcomes are PROCESS-wide (shared by every HipGemm, seeded from the plan):
        # two models / trainers in one process must not pick different kernels -- and
        # so different summation orders -- for the same shape
        if not _RACES:
            _RACES["tn"] = dict(_PINNED["tn"])
            _RACES["splitk"] = dict(_PINNED["splitk"])
        self._choice = _RACES["tn"]  # (M, N, K) -> "bf16" | None (library); (kind, M, N, K) -> bool (fused)
        self._race = os.environ.get("DLT_GEMM_TN", "1") != "0"
        self._splitk = _RACES["splitk"]  # wgrad (M, N, K) -> token slices (1 = plain accumulate GEMM)
        self._splitk_on = os.environ.get("DLT_WGRAD_SPLITK", "1") != "0"
        self._hand_wgrad = os.environ.get("DLT_WGRAD_HAND", "1") != "0"
        self._fuse = os.environ.get("DLT_GEMM_FUSED", "1") != "0"
        self._dgrad_on = os.environ.get("DLT_GEMM_DGRAD", "1") != "0"
        # fp16 activations on the hand-written forward (the plan's shape pins) and fused
        # down-dgrad + SwiGLU-backward kernels (both instantiated for IEEE half and
        # tested): DLT_GEMM_FP16_HAND=1 ("fwd" / "dswiglu": only one of the two).  Off by
        # default: --precision fp16 steps measured 744-749k with them vs 744-756k on
        # hipBLASLt + the unfused SwiGLU backward (r5_fp16hand.sh in tools/ab/README.md, same box)
        _f16 = os.environ.get("DLT_GEMM_FP16_HAND", "0")
        self._fp16_hand = _f16 in ("1", "fwd")
        self._fp16_dswiglu = _f16 in ("1", "dswiglu")
        _INSTANCES.append(weakref.ref(self))

    def _lib_linear(self, x, w, y):
        M, K = x.shape
        N = w.shape[0]
        _gemm(1, 0, N, M, K, w, _rowmajor(w), x, _rowmajor(x), y, N)

    @staticmethod
    def _hand_ok(*ts) -> bool:
        """Operands the hand-written kernels take (race outcomes are keyed by shape only,
        so a dtype check must precede every cached hand-written pick)."""
        return all(t.dtype == torch.bfloat16 and t.is_contiguous() for t in ts)

    @staticmethod
    def _hand16_ok(*ts) -> bool:
        """Operands of the kernels instantiated for both 16-bit formats (the data-gradient
        GEMM): all bf16 or all fp16, contiguous."""
        return (ts[0].dtype in (torch.bfloat16, torch.float16)
                and all(t.dtype == ts[0].dtype and t.is_contiguous() for t in ts))

    @staticmethod
    def _wgrad_hand_ok(dy, x, to16: bool = False) -> bool:
        """Operands the hand-written weight-gradient kernels take: bf16 or fp16, one format
        (the kernels are instantiated for both; the 16-bit-output route sums its fp32
        partials into the operands' format with hip.splitk_sum_bf16, which takes both)."""
        ok = dy.dtype == x.dtype and dy.is_contiguous() and x.is_contiguous()
        return ok and dy.dtype in (torch.bfloat16, torch.float16)

    def _can_race(self, x, w, dtypes=(torch.bfloat16,)) -> bool:
        return (self._race and x.is_contiguous() and w.is_contiguous() and x.dtype in dtypes
                and w.dtype == x.dtype and not torch.cuda.is_current_stream_capturing())

    def _pick(self, x, w, y):
        """Forward projection race, once per shape: hipBLASLt (None), the persistent
        hand-written kernel ("bf16") or the one-tile-per-workgroup one ("fw4"); a hand-written pick
        must beat the library by RACE_MARGIN.  The shipped plan pins the in-step winners."""
        from . import hip
        key = (x.shape[0], w.shape[0], x.shape[1])
        if key in self._choice:
            return self._choice[key]
        if not self._can_race(x, w):
            return None  # not recorded: decided when a bf16 call can race (fp16 replays pins)
        choice = None
        t_lib = _time_of(lambda: self._lib_linear(x, w, y))
        best = self.RACE_MARGIN * t_lib
        cands = []
        if hip.gemm_bf16_fits(*key):
            cands.append(("bf16", lambda: hip.gemm_bf16(x, w, out=y)))
        if hip.gemm_fw4_fits(*key):
            cands.append(("fw4", lambda: hip.gemm_fw4(x, w, out=y)))
        for name, fn in cands:
            t = _time_of(fn)
            if t < best:
                best, choice = t, name
        self._choice[key] = choice
        return choice

    def linear(self, x: torch.Tensor, w: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
        M, K = x.shape
        N = w.shape[0]
        if out is not None and (out.shape != (M, N) or not out.is_contiguous() or out.dtype != x.dtype):
            raise ValueError("linear: out must be a contiguous [M, N] tensor of the input dtype")
        y = torch.empty(M, N, dtype=x.dtype, device=x.device) if out is None else out
        pick = self._pick(x, w, y) if self._race and self._hand16_ok(x, w) else None
        from . import hip
        if pick == "bf16" and (x.dtype == torch.bfloat16 or self._fp16_hand) and hip.gemm_bf16(x, w, out=y) is not None:
            return y
        if pick == "fw4" and hip.gemm_fw4(x, w, out=y) is not None:
            return y
        if isinstance(pick, str) and pick.startswith("fw4:") and hip.gemm_fw4(x, w, out=y, flags=int(pick[4:])) is not None:
            return y  # "fw4:<flags>": the kernel with its own launch flags (schedule / store flavour)
        self._lib_linear(x, w, y)
        return y

    def _fused_pick(self, kind, x, w, fused, unfused, key=None) -> bool:
        """Race a hand-written kernel (``fused``) against its library equivalent once
        per key; kinds "rope" / "swiglu" / "dswiglu" are fused epilogues
        (``DLT_GEMM_FUSED=0`` turns them off), "dgrad" the plain data-gradient GEMM."""
        plain = kind.startswith("dgrad")  # the data-gradient kernel (bf16 and fp16 instances)
        both16 = plain or kind == "dswiglu16"  # kernels instantiated for both 16-bit formats
        on = self._fuse if not plain else True
        if not (on and (self._hand16_ok(x, w) if both16 else self._hand_ok(x, w))):
            return False
        key = key or (kind, x.shape[0], w.shape[0], x.shape[1])
        choice = self._choice.get(key)
        if choice is None:
            if not self._can_race(x, w, (torch.bfloat16, torch.float16) if both16 else (torch.bfloat16,)):
                return False  # not recorded: decided again when racing is possible
            choice = _time_of(fused, inner=3) < self.RACE_MARGIN * _time_of(unfused, inner=3)
            self._choice[key] = choice
        return bool(choice)

    def linear_rope(self, x: torch.Tensor, w: torch.Tensor, B: int, S: int, nh: int, cos: torch.Tensor,
                    sin: torch.Tensor, ops) -> torch.Tensor:
        """qkv = x @ Wqkv^T with RoPE applied in place to the q and k heads (the packed
        layout the attention kernels read): the fused hand-written GEMM or the linear +
        ``ops.rope_qk_inplace`` pair, whichever ran faster when the shape was first seen."""
        from . import hip
        M = x.shape[0]
        y = torch.empty(M, w.shape[0], dtype=x.dtype, device=x.device)

        def unfused():
            self.linear(x, w, out=y)
            ops.rope_qk_inplace(y, B, S, nh, cos, sin)

        def fused():
            hip.gemm_qkv_rope(x, w, S, cos, sin, out=y)
        ok = (w.shape[0] == 3 * nh * 64 and hip.gemm_bf16_fits192(M, w.shape[0], x.shape[1]) and M % S == 0
              and cos.dtype == torch.float32 and cos.is_contiguous() and sin.is_contiguous())
        if ok and self._fused_pick("rope", x, w, fused, unfused):
            fused()
        else:
            unfused()
        return y

    def linear_swiglu(self, x: torch.Tensor, w: torch.Tensor, ops, s_out: torch.Tensor = None):
        """(gu, s): gu = x @ Wgu^T and s = silu(gate) * up, fused in the GEMM epilogue or
        as linear + ``ops.swiglu_fwd`` (raced once per shape like :meth:`linear`)."""
        from . import hip
        M = x.shape[0]
        I2 = w.shape[0]
        gu = torch.empty(M, I2, dtype=x.dtype, device=x.device)
        s = torch.empty(M, I2 // 2, dtype=x.dtype, device=x.device) if s_out is None else s_out

        def unfused():
            self.linear(x, w, out=gu)
            ops.swiglu_fwd(gu, out=s)

        def fused():
            hip.gemm_gu_swiglu(x, w, gu_out=gu, s_out=s)
        # the 4-wave k_gemm_fw4 with the SwiGLU epilogue: plan kind "swiglu4" (its launch flags)
        # or DLT_GEMM_FW4_SWIGLU=<flags> (A/B knob)
        fw4 = os.environ.get("DLT_GEMM_FW4_SWIGLU") or self._choice.get(("swiglu4", M, I2, x.shape[1]))
        if fw4 is not None and self._hand16_ok(x, w) and s.is_contiguous() and \
                hip.gemm_fw4_swiglu(x, w, gu_out=gu, s_out=s, flags=int(fw4)) is not None:
            return gu, s
        ok = I2 % 192 == 0 and hip.gemm_bf16_fits192(M, I2, x.shape[1]) and s.is_contiguous()
        if ok and self._fused_pick("swiglu", x, w, fused, unfused):
            fused()
        else:
            unfused()
        return gu, s

    def report_choices(self) -> dict:
        names = {"bf16": "hand-written gemm_bf16 (persistent)", "fw4": "hand-written gemm_fw4"}
        out = {f"M{k[0]}xN{k[1]}xK{k[2]}": ("hipBLASLt" if c is None else names.get(c, f"hand-written gemm_{c}"))
               for k, c in self._choice.items() if len(k) == 3}
        out.update({f"{k[0]} M{k[1]}xN{k[2]}xK{k[3]}": (("hand-written gemm_dgrad" if c else "hipBLASLt")
                                                       if k[0].startswith("dgrad") else
                                                       (f"fused gemm_fw4 (flags {c})" if c is not None else "not used")
                                                       if k[0] == "swiglu4" else
                                                       ("fused gemm_bf16" if c else "unfused (linear + kernel)"))
                    for k, c in self._choice.items() if len(k) == 4})
        out.update({f"wgrad{f' ({key[3]} out)' if len(key) == 4 else ''} M{key[0]}xN{key[1]}xK{key[2]}":
                    ("hand-written gemm_wgrad stream-K" if s == self.STREAMK else
                     f"hand-written gemm_wgrad x{-s}" if s < 0 else
                     f"hipBLASLt split-K x{s}" if s > 1 else "hipBLASLt plain")
                    for key, s in self._splitk.items()})
        return out

    def _lib_dgrad(self, dy, w, dx):
        M, N = dy.shape
        K = w.shape[1]
        _gemm(0, 0, K, M, N, w, _rowmajor(w), dy, _rowmajor(dy), dx, K)

    def linear_dgrad(self, dy: torch.Tensor, w: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
        """dX[M, K] = dY[M, N] @ W[N, K]: the hand-written reduction-major-B kernel
        (``hip.gemm_dgrad``, W read as stored) or hipBLASLt, raced once per shape (kind
        "dgrad" in the plan's "fused" table; ``DLT_GEMM_DGRAD=0``: library only)."""
        from . import hip
        M, N = dy.shape
        K = w.shape[1]
        dx = torch.empty(M, K, dtype=dy.dtype, device=dy.device) if out is None else out
        ok = self._dgrad_on and self._race and hip.gemm_bf16_fits(M, K, N) and self._hand16_ok(dy, w, dx)
        # bf16 and fp16 race separately (kind "dgrad" / "dgrad16"): one format's pick must
        # not decide the other's
        kind = "dgrad" if dy.dtype == torch.bfloat16 else "dgrad16"
        if ok and self._fused_pick(kind, dy, w, lambda: hip.gemm_dgrad(dy, w, out=dx),
                                   lambda: self._lib_dgrad(dy, w, dx), key=(kind, M, K, N)):
            hip.gemm_dgrad(dy, w, out=dx)
        else:
            self._lib_dgrad(dy, w, dx)
        return dx

    def linear_dgrad_swiglu(self, dd: torch.Tensor, wdown: torch.Tensor, gu: torch.Tensor, ops,
                            out: torch.Tensor = None, s_out: torch.Tensor = None) -> torch.Tensor:
        """dgu[M, 2I]: the down projection's data gradient ds = dd @ Wdown and the SwiGLU
        backward against the kept gu, fused in one hand-written kernel
        (``hip.gemm_down_swiglu_bwd``) or as ``linear_dgrad`` + ``ops.swiglu_bwd`` --
        raced once per shape (kind "dswiglu").  ``s_out``: also (re)writes the SwiGLU
        output s = silu(g) * u there (the forward's bits; engine s ring)."""
        from . import hip
        M, H = dd.shape
        I = wdown.shape[1]
        dgu = torch.empty(M, 2 * I, dtype=dd.dtype, device=dd.device) if out is None else out

        def unfused():
            ds = self.linear_dgrad(dd, wdown)
            if s_out is not None:
                ops.swiglu_bwd(gu, ds, out=dgu, s_out=s_out)
            else:
                ops.swiglu_bwd(gu, ds, out=dgu)

        def fused():
            hip.gemm_down_swiglu_bwd(dd, wdown, gu, out=dgu, s_out=s_out)
        # bf16 and fp16 race separately (kind "dswiglu" / "dswiglu16")
        kind = "dswiglu" if dd.dtype == torch.bfloat16 else "dswiglu16"
        ok = (self._dgrad_on and self._race and hip.gemm_bf16_fits192(M, I, H) and tuple(gu.shape) == (M, 2 * I)
              and (dd.dtype == torch.bfloat16 or self._fp16_dswiglu)
              and self._hand16_ok(dd, wdown, gu, dgu, *(() if s_out is None else (s_out,))))
        if ok and self._fused_pick(kind, dd, wdown, fused, unfused, key=(kind, M, I, H)):
            fused()
        else:
            unfused()
        return dgu

    @staticmethod
    def _wgrad_plain(dw2, dy, x):
        M, N = dy.shape
        K = x.shape[1]
        _gemm(0, 1, K, N, M, x, _rowmajor(x), dy, _rowmajor(dy), dw2, K, 1.0, 1.0)

    @staticmethod
    def _wgrad_split(dw2, dy, x, s):
        """Split-K over tokens: s strided-batched GEMMs (slice i = rows [i*M/s, (i+1)*M/s))
        into an fp32 [s, N, K] scratch, then one fixed-order sum into dw (hip.splitk_acc).
        The skinny wgrads (768x768, 768x2304 outputs, K = 32768 tokens) have too few
        output tiles for 256 CUs; slicing K multiplies the tile count by s."""
        from . import hip
        M, N = dy.shape
        K = x.shape[1]
        ms = M // s
        lx, ly = _rowmajor(x), _rowmajor(dy)
        part = torch.empty(s, N, K, dtype=torch.float32, device=dw2.device)
        _gemm_batched(0, 1, K, N, ms, x, lx, ms * lx, dy, ly, ms * ly, part, K, N * K, s, 1.0, 0.0)
        hip.splitk_acc(part, dw2)

    @staticmethod
    def _wgrad_hand(dw2, dy, x, s, to_bf16=False):
        """The hand-written 256 x 192 MFMA weight-gradient kernel (csrc/gemm_wgrad.hip)
        with s token splits.  fp32 dw2: accumulated in place (s = 1) or partials + one
        fixed-order sum; bf16 dw2 (wgrad_set): partials summed straight into bf16."""
        from . import hip
        M, N = dy.shape
        K = x.shape[1]
        if not to_bf16:
            if not hip.gemm_wgrad(dw2, dy, x, s):
                raise RuntimeError(f"hand wgrad cannot tile {M}x{N}x{K}")
            return
        part = torch.empty(s, N, K, dtype=torch.float32, device=dw2.device)
        if s == 1:
            part.zero_()
            ok = hip.gemm_wgrad(part[0], dy, x, 1)
        else:
            ok = hip.gemm_wgrad(None, dy, x, s, part=part)  # partials only
        if not ok:
            raise RuntimeError(f"hand wgrad cannot tile {M}x{N}x{K}")
        hip.splitk_sum_bf16(part, dw2)

    # splitk plan value of the stream-K hand-written weight gradient (hip.gemm_wgrad_sk)
    STREAMK = -1024

    def _run_wgrad(self, dw2, dy, x, s, to_bf16):
        """One weight-gradient route: s = 1 hipBLASLt plain (beta 1 into fp32, or beta 0
        with a bf16 D), s > 1 hipBLASLt split-K, s < 0 the hand-written kernel with -s
        splits; bf16 outputs take the fp32 partials summed straight into bf16."""
        from . import hip
        M, N = dy.shape
        K = x.shape[1]
        if s == self.STREAMK and not to_bf16:
            if not hip.gemm_wgrad_sk(dw2, dy, x):
                raise RuntimeError(f"stream-K wgrad cannot tile {M}x{N}x{K}")
        elif s < 0:
            self._wgrad_hand(dw2, dy, x, -s if s != self.STREAMK else 8, to_bf16=to_bf16)
        elif s > 1 and to_bf16:
            ms = M // s
            lx, ly = _rowmajor(x), _rowmajor(dy)
            part = torch.empty(s, N, K, dtype=torch.float32, device=dw2.device)
            _gemm_batched(0, 1, K, N, ms, x, lx, ms * lx, dy, ly, ms * ly, part, K, N * K, s, 1.0, 0.0)
            hip.splitk_sum_bf16(part, dw2)
        elif s > 1:
            self._wgrad_split(dw2, dy, x, s)
        elif to_bf16:
            _gemm(0, 1, K, N, M, x, _rowmajor(x), dy, _rowmajor(dy), dw2, K, 1.0, 0.0)
        else:
            self._wgrad_plain(dw2, dy, x)

    def _pick_splitk(self, dw2, dy, x, to_bf16=False):
        """Weight-gradient race, per (M, N, K) and output dtype: hipBLASLt plain (1) /
        hipBLASLt split-K (s > 1) / the hand-written kernel with s splits (-s).  The
        bf16-output routes (wgrad_set) race separately, key (M, N, K, "bf16"): the
        library's bf16-D kernels are different (and slower) ones.  Recorded in the plan."""
        from . import hip
        M, N = dy.shape
        K = x.shape[1]
        # 16-bit outputs race per format ("bf16" / "fp16" key suffix)
        key = (M, N, K, "bf16" if dw2.dtype == torch.bfloat16 else "fp16") if to_bf16 else (M, N, K)
        if key in self._splitk:
            return self._splitk[key]
        # library split-K: skinny outputs only (its [s, N, K] fp32 scratch)
        cands = [s for s in self.SPLITK_CANDIDATES if M % (s * 8) == 0 and (N * K) % 4 == 0
                 and N * K <= 4096 * 4096]
        hand = self._hand_wgrad and self._wgrad_hand_ok(dy, x, to_bf16) and hip.wgrad_fits(M, N, K)
        if hand:  # whole rounds of 256 workgroups, plus a few fixed depths (sweep in
            # profiles/r3_wgrad.md: the best split is shape-specific, 5..16 here); the
            # split partials ([s, N, K] fp32) stay under ~1 GB
            tiles = ((N + 255) // 256) * (K // hip.wgrad_bn(K))
            hs = {max(1, (256 * r) // tiles) for r in (1, 2, 3)} | {2, 3, 4, 8, 16}
            cands += [-h for h in sorted(hs) if h <= min(64, M // 128) and (h == 1 or h * N * K * 4 <= 1 << 30)]
            if not to_bf16:  # stream-K (fp32 accumulate only)
                cands.append(self.STREAMK)
        if (not (self._splitk_on or hand) or not cands or torch.cuda.is_current_stream_capturing()):
            self._splitk[key] = 1
            return 1
        # timing must not disturb the real accumulator / gradient buffer
        scratch = torch.zeros(N, K, dtype=dw2.dtype, device=dy.device)

        def t_of(fn):
            fn()
            torch.cuda.synchronize()
            best = float("inf")
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(3):
                    fn()
                e1.record()
                e1.synchronize()
                best = min(best, e0.elapsed_time(e1))
            return best
        best, choice = t_of(lambda: self._run_wgrad(scratch, dy, x, 1, to_bf16)), 1
        for s in cands:
            if s > 1 and not self._splitk_on:
                continue
            t = t_of(lambda: self._run_wgrad(scratch, dy, x, s, to_bf16))
            if t < (self.RACE_MARGIN if s < 0 else 0.93) * best:
                best, choice = t, s
        del scratch
        self._splitk[key] = choice
        return choice

    def _resolve(self, s, dy, x, to16=False):
        """A recorded hand-written pick (-s) falls back to the library when the operands
        do not suit the kernel or DLT_WGRAD_HAND=0: split-K x s if the tokens divide,
        else the plain accumulate GEMM."""
        if s < 0 and not (self._hand_wgrad and self._wgrad_hand_ok(dy, x, to16)):
            s = -s if self._splitk_on and -s in self.SPLITK_CANDIDATES and dy.shape[0] % (-s * 8) == 0 else 1
        return s

    def wgrad_set(self, dw: torch.Tensor, dy: torch.Tensor, x: torch.Tensor) -> None:
        """dw (bf16, overwritten) = dy^T @ x: a weight gradient written straight in the
        reduce dtype (the FSDP runtime's per-micro-step send buffer): the raced bf16 route
        (library GEMM with beta = 0 and a bf16 D, or split-K / hand-written partials
        summed into bf16 in fixed order)."""
        M, N = dy.shape
        K = x.shape[1]
        dw2 = dw.view(N, K)
        if dw2.dtype not in (torch.bfloat16, torch.float16) or dw2.dtype != dy.dtype or not dw2.is_contiguous():
            raise ValueError("wgrad_set output must be contiguous bf16 / fp16 (the operands' dtype)")
        s = self._resolve(self._pick_splitk(dw2, dy, x, to_bf16=True), dy, x, True)
        self._run_wgrad(dw2, dy, x, s, True)

    def wgrad_acc(self, dw: torch.Tensor, dy: torch.Tensor, x: torch.Tensor) -> None:
        """dw (fp32) += dy^T @ x.  A bf16 ``dw`` is refused: overwriting is ``wgrad_set``'s
        contract, and silently switching to it would drop an earlier contribution."""
        if dw.dtype in (torch.bfloat16, torch.float16):
            raise ValueError("wgrad_acc accumulates into fp32; use wgrad_set for a 16-bit gradient")
        M, N = dy.shape
        K = x.shape[1]
        dw2 = dw.view(N, K)
        if dw2.dtype != torch.float32 or not dw2.is_contiguous():
            raise ValueError("wgrad accumulator must be contiguous fp32")
        s = self._resolve(self._pick_splitk(dw2, dy, x), dy, x)
        self._run_wgrad(dw2, dy, x, s, False)
