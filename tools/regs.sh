#!/bin/bash
# Register / scratch usage per kernel of one translation unit (developer tool):
#   bash tools/regs.sh svdsolver_amd/csrc/brd_blk_cqr.hip [kernel-name-filter]
f=$1; pat=${2:-.}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$(dirname $0)/../include -I$(dirname $0)/../svdsolver_amd/csrc \
  --cuda-device-only -c "$f" -o /tmp/_regs.o -Rpass-analysis=kernel-resource-usage 2>&1 \
  | grep -E "Function Name|VGPRs:|AGPRs|ScratchSize|SGPRs:" | paste - - - - - \
  | sed 's/remark: //g;s/\[-Rpass-analysis=kernel-resource-usage\]//g;s#[^ ]*\.hip:[0-9]*:[0-9]*:##g;s/Function Name: //;s/  */ /g' \
  | grep -E "$pat"
