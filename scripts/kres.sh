#!/bin/bash
# Register / LDS / spill figures of the gfx950 kernels in a built object whose
# (mangled) name matches a pattern:  bash scripts/kres.sh build/lte_kernels.o k_rx_frame_w
set -e
O=$1; PAT=$2
B=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
$B/llvm-objcopy --dump-section=.hip_fatbin="$T/fat.bin" "$O" "$T/copy.o"   # (without an output file objcopy rewrites $O)
$B/clang-offload-bundler --unbundle --type=o --input="$T/fat.bin" --targets=hipv4-amdgcn-amd-amdhsa--gfx950 \
  --output="$T/k.co"
$B/llvm-readelf --notes "$T/k.co" | python3 -c '
import re, sys
pat = sys.argv[1]
txt = sys.stdin.read()
for blk in re.split(r"\n\s+- \.agpr_count", txt)[1:]:
    blk = ".agpr_count" + blk
    m = re.search(r"\.name:\s+(\S+)", blk)
    if not m or pat not in m.group(1):
        continue
    f = {k: re.search(r"\.%s:\s+(\S+)" % k, blk) for k in
         ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
          "group_segment_fixed_size", "private_segment_fixed_size")}
    print(m.group(1)[:90], " ".join("%s=%s" % (k, v.group(1)) for k, v in f.items() if v))
' "$PAT"
rm -rf "$T"
