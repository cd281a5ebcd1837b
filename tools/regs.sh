#!/bin/bash
# Register / LDS / spill report of the device kernels (compile only, no GPU):
#   tools/regs.sh [kernel-name-regex] [extra hipcc flags, e.g. -DYK_SHADOW_WAVES=6]
here="$(cd "$(dirname "$0")" && pwd)"
cd "$here/../core_amd"
pat=${1:-k_trace}
shift
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math \
  -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-rdc --cuda-device-only -c -o /dev/null csrc/yk_device.hip \
  -Rpass-analysis=kernel-resource-usage "$@" 2>&1 | python3 "$here/regs_parse.py" "$pat"
