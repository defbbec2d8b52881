#!/bin/bash
# Build ops/_dlt_kernels_base.so from the kernel sources of git revision $1 (default HEAD)
# for tools/ab/kernels_ab.sh (extra hipcc flags, e.g. a diagnostic -D, in DLT_BASE_CFLAGS).  Runs on the CPU container (hipcc cross-compiles gfx950).
set -eu
rev=${1:-HEAD}
mkdir -p .scratch && tmp=$(mktemp -d -p "$PWD/.scratch")
git archive "$rev" distributed_llm_trainer_amd/ops/csrc | tar -x -C "$tmp"
objs=()
for f in "$tmp"/distributed_llm_trainer_amd/ops/csrc/*.hip; do
  o="$tmp/$(basename "$f" .hip).o"
  /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wno-unused-result -mllvm -amdgpu-mfma-vgpr-form ${DLT_BASE_CFLAGS:-} \
    -I "$tmp/distributed_llm_trainer_amd/ops/csrc" -c "$f" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o distributed_llm_trainer_amd/ops/_dlt_kernels_base.so "${objs[@]}"
rm -rf "$tmp"
echo "built ops/_dlt_kernels_base.so from $rev"
