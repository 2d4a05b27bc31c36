#!/bin/bash
# Build libcsa_kernels.so from the kernel sources of a git revision into ab/<name>/ (an A/B
# baseline for same-box comparisons: CSA_KERNEL_LIB=ab/<name>/libcsa_kernels.so).
# usage: scripts/build_variant.sh <rev> <name>
set -euo pipefail
rev=$1; name=$2
root=$(git rev-parse --show-toplevel)
src=$(mktemp -d)
out=$root/ab/$name
mkdir -p "$out" "$src/kernels" "$src/comm"
for f in $(git -C "$root" ls-tree --name-only "$rev" cloud_server_amd/csrc/kernels/ cloud_server_amd/csrc/comm/); do
  git -C "$root" show "$rev:$f" > "$src/$(basename "$(dirname "$f")")/$(basename "$f")"
done
objs=()
for f in "$src"/kernels/*.hip "$src"/comm/*.hip; do
  o="$src/$(basename "$f").o"
  /opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -std=c++17 -ffp-contract=fast-honor-pragmas \
    -Wno-unused-result -I"$src/kernels" -I"$src/comm" -c "$f" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 "${objs[@]}" -o "$out/libcsa_kernels.so"
echo "$rev" > "$out/REV"
rm -rf "$src"
echo "$out/libcsa_kernels.so"
