#!/bin/bash
# HBM ceiling by read:write mix (tools/stream_mix.hip), at 288 MiB and 1152 MiB moved per launch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-stream_mix}; mkdir -p $O
[ -x tools/bin/stream_mix ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/stream_mix.hip -o tools/bin/stream_mix || exit 1
timeout -k 10 120 tools/bin/stream_mix 288 5 > $O/stream_mix_288MiB.txt 2>&1
rc=$?; echo "stream_mix 288 rc=$rc"; cat $O/stream_mix_288MiB.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 tools/bin/stream_mix 1152 3 > $O/stream_mix_1152MiB.txt 2>&1
rc=$?; echo "stream_mix 1152 rc=$rc"; cat $O/stream_mix_1152MiB.txt
exit $rc
