"""Write a variant of the shipped GEMM plan with some picks overridden (for same-box A/Bs).

usage: python tools/ab/plan_variant.py OUT.json [table:key=value ...]
  table: tn | fused | splitk;  value: null / true / false / an int / a string
  e.g.  tn:16384x768x768=bf16 tn:16384x50304x768=fwd fused:dswiglu:16384x3072x768=false
  the shorthand  fwd=VALUE  sets every M=16384 forward role except qkv (o, gate/up, down,
  lm_head) to VALUE; allfwd=VALUE includes qkv.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FWD = ("16384x768x768", "16384x6144x768", "16384x768x3072", "16384x50304x768")


def _val(s):
    if s == "null":
        return None
    if s in ("true", "false"):
        return s == "true"
    try:
        return int(s)
    except ValueError:
        return s


def main(argv):
    out, edits = argv[0], argv[1:]
    with open(os.path.join(ROOT, "configs", "gemm_plan_mi355x.json")) as f:
        plan = json.load(f)
    for e in edits:
        lhs, rhs = e.split("=", 1)
        if lhs in ("fwd", "allfwd"):
            for k in FWD + (("16384x2304x768",) if lhs == "allfwd" else ()):
                plan["tn"][k] = _val(rhs)
            continue
        table, key = lhs.split(":", 1)
        plan[table][key] = _val(rhs)
    with open(out, "w") as f:
        json.dump(plan, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1:])
