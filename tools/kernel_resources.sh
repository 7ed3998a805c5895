#!/usr/bin/env bash
# usage: tools/kernel_resources.sh <object.hip.o> [name-regex]
# VGPR / SGPR / LDS / scratch per kernel of a built object's gfx950 code object
# (the AMDGPU metadata notes), e.g. tools/kernel_resources.sh \
#   gaussian_splatting_with_eye_tracking_amd/_build/backward.hip.o render_bwd
set -eu
obj=$1; pat=${2:-.}
d=$(mktemp -d)
trap 'rm -rf "$d"' EXIT
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section .hip_fatbin="$d/fb" "$obj"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input="$d/fb" \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="$d/co" >/dev/null
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$d/co" > "$d/notes"
python3 - "$pat" "$d/notes" <<'PY'
import re, sys
pat = re.compile(sys.argv[1])
txt = open(sys.argv[2]).read()
def g(blk, k):
    m = re.search(r"\." + k + r":\s+(\d+)", blk)
    return m.group(1) if m else "?"
for blk in txt.split("- .agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk).group(1)
    if pat.search(name):
        print("vgpr %4s sgpr %4s lds %6s scratch %4s spill %3s  %s" % (
            g(blk, "vgpr_count"), g(blk, "sgpr_count"), g(blk, "group_segment_fixed_size"),
            g(blk, "private_segment_fixed_size"), g(blk, "vgpr_spill_count"), name))
PY
