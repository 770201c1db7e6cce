#!/bin/bash
# Register / scratch / LDS report of one HIP source, optionally with an occupancy target:
#   tools/kres.sh fet-ode_amd/csrc/fetode_bwd.hip [waves_per_eu] [kernel-name-filter]
src=$1; w=${2:-0}; filt=${3:-.}
dir=$(dirname "$src")
tmp="$dir/.kres_$$.hip"
if [ "$w" = 0 ]; then cp "$src" "$tmp"; else
  sed "s/__launch_bounds__(\([^)]*\)) void/__launch_bounds__(\1) __attribute__((amdgpu_waves_per_eu($w, $w))) void/" "$src" > "$tmp"; fi
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -Wall -Wno-unused-function $KRES_FLAGS \
  -c -o /tmp/kres_$$.o "$tmp" -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "error|Function Name|VGPRs:|Spill|ScratchSize|Occupancy|LDS Size" | sed 's/.*remark: *//' |
  awk -v f="$filt" '/Function Name/ {show = ($0 ~ f)} show || /error/'
rm -f "$tmp" /tmp/kres_$$.o
