#!/bin/bash
# Occupancy caps on the many-stream mixes (tools/stream_mix.hip occ), 288 MiB moved per launch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-stream_mix}; mkdir -p $O
timeout -k 10 150 tools/bin/stream_mix 288 5 occ > $O/stream_occ_288MiB.txt 2>&1
rc=$?; echo "stream_mix occ rc=$rc"; cat $O/stream_occ_288MiB.txt
exit $rc
