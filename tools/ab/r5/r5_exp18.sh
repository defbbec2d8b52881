# round 5 batch 18: private norm gradients (no per-block wait) vs per-block wait; head share
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
VARIANTS="priv:DLT_X=0 nopriv:DLT_PRIV_NORM=0 noshare:DLT_HEAD_SHARE=0" REPS=3 bash tools/ab/env_ab.sh
