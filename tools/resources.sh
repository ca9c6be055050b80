#!/bin/bash
# Register / spill / LDS report of the engine's kernels (hipcc kernel-resource-usage remarks).
#   tools/resources.sh [name-filter] [extra hipcc flags...]
R=$(cd "$(dirname "$0")/.." && pwd)
F=${1:-}
shift || true
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result \
    -Rpass-analysis=kernel-resource-usage "$@" -o /tmp/gd_res.so "$R/galaxy-deconv_amd/csrc/gd_engine.hip" \
    > /tmp/gd_res.txt 2>&1
grep -i " error" /tmp/gd_res.txt | head
python3 "$R/tools/resource_report.py" "$F" < /tmp/gd_res.txt
