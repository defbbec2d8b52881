"""Build-time ISA checks on the gfx950 kernels (CPU: hipcc cross-compiles to assembly).

The attention forward / dQ kernels read K/V row fragments through inline-asm
``ds_read_b128`` and retire them with a COUNTED ``s_waitcnt lgkmcnt(4)``
(``ops/csrc/attention.hip`` ``lgkm_wait4``).  That count is only sound while every
lgkm-counted operation in flight is an LDS access (LDS returns in issue order); a
scalar-memory load (``s_load*`` / ``s_buffer_load*`` / ``s_memtime``) returns out of
order, and one issued inside the counted window would let the wait retire the wrong
fragments.  Nothing in the source pins the compiler's placement of SMEM loads, so this
test reads the emitted assembly: between every counted ``lgkmcnt(N > 0)`` wait and the
last ``lgkmcnt(0)`` before it there must be no SMEM instruction.
"""
import os
import re
import shutil
import subprocess

import pytest

from distributed_llm_trainer_amd.ops import build as kbuild

SMEM = ("s_load", "s_buffer_load", "s_memtime", "s_memrealtime", "s_scratch_load", "s_atc_probe")


def _device_asm(src: str, tmp_path, extra=()):
    hipcc = kbuild.hipcc()
    out = tmp_path / (os.path.basename(src) + ".s")
    flags = [f for f in kbuild.CXXFLAGS if f != "-fPIC"]
    cmd = [hipcc, *flags, *extra, "--cuda-device-only", "-S", "-I", kbuild.CSRC, src, "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return out.read_text()


def _counted_lgkm_violations(asm: str):
    ins = [ln.strip() for ln in asm.split("\n")
           if ln.startswith("\t") and not ln.strip().startswith((".", ";"))]
    counted, bad = 0, []
    for k, t in enumerate(ins):
        m = re.match(r"s_waitcnt\b.*lgkmcnt\((\d+)\)", t)
        if not m or m.group(1) == "0":
            continue
        counted += 1
        for j in range(k - 1, -1, -1):
            u = ins[j]
            if u.startswith("s_waitcnt") and "lgkmcnt(0)" in u:
                break
            if u.startswith("s_endpgm"):
                break
            if u.startswith(SMEM):
                bad.append((k, u))
                break
    return counted, bad


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not available")
@pytest.mark.parametrize("kread_asm", ["1", "0"])
def test_attention_counted_lds_waits_have_no_smem_in_flight(tmp_path, kread_asm):
    src = os.path.join(kbuild.CSRC, "attention.hip")
    asm = _device_asm(src, tmp_path, ("-DDLT_ATTN_KREAD_ASM=" + kread_asm,))
    counted, bad = _counted_lgkm_violations(asm)
    if kread_asm == "1":
        assert asm.count("lgkmcnt(4)") > 0, "the asm K-row reads' counted wait is gone"
    assert counted > 0
    assert not bad, f"SMEM load inside a counted LDS wait window: {bad[:5]}"


def _kernel_bodies(asm: str, pattern: str):
    """name -> instruction lines of every kernel whose symbol matches ``pattern``."""
    lines = asm.split("\n")
    out = {}
    for i, ln in enumerate(lines):
        m = re.match(r"^(_Z\w+):", ln)
        if m and re.search(pattern, m.group(1)):
            j = i + 1
            while j < len(lines) and not lines[j].startswith(".Lfunc_end"):
                j += 1
            out[m.group(1)] = [t.strip() for t in lines[i + 1:j] if t.startswith("\t")]
    return out


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not available")
@pytest.mark.parametrize("src,pattern", [("gemm_wgrad.hip", r"k_gemm_wgrad"),
                                         ("gemm_bf16.hip", r"k_gemm_bf16ILi192ELi0ELb1ELi")])
def test_gemm_operand_format_instantiations_use_their_mfma(tmp_path, src, pattern):
    """The weight- and data-gradient GEMMs are instantiated per 16-bit operand format
    (template HK: 0 = bf16, 1 = fp16).  Each instantiation must issue only its own MFMA
    (v_mfma_f32_16x16x32_bf16 / _f16) -- a mix-up would run fp16 bits through the bf16
    datapath (or the reverse) without any shape error."""
    asm = _device_asm(os.path.join(kbuild.CSRC, src), tmp_path)
    bodies = _kernel_bodies(asm, pattern)
    # HK: the first int template argument of k_gemm_wgrad<HK, BN>, the last int one of
    # k_gemm_bf16<BN, EPI, BT, HK, LATE> (a bool LATE after it)
    pick = 0 if "wgrad" in pattern else -1
    hk = {k: re.findall(r"Li(\d+)E", k)[pick] for k in bodies}
    assert set(hk.values()) == {"0", "1"}, sorted(bodies)
    for name, ins in bodies.items():
        fmt = "f16" if hk[name] == "1" else "bf16"
        other = "bf16" if fmt == "f16" else "f16"
        mf = [t for t in ins if t.startswith("v_mfma")]
        assert mf, name
        assert all(f"x32_{fmt} " in t for t in mf), (name, [t for t in mf if f"x32_{fmt} " not in t][:3])
        assert not any(f"x32_{other} " in t for t in mf), name
