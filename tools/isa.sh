#!/bin/bash
# Device assembly of ONE qconv_glds_kernel instance (fast: no other instantiation).
#   tools/isa.sh "3,1,1,4,8,1,2,false,2,64,true,false,true" out.s
set -e
D=$(cd "$(dirname "$0")/.." && pwd)/semilayer-wise-mixed-precision-quantization_amd/csrc
T=$(mktemp /tmp/isa_XXXX.hip)
cat > "$T" <<EOS
#include "$D/conv_glds_kernel.h"
namespace smpq { template __global__ void qconv_glds_kernel<$1>(ConvArgs); }
EOS
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off --cuda-device-only -S "$T" -o "$2" ${@:3}
rm -f "$T"
