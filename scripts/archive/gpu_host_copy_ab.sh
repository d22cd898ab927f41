#!/bin/bash
# host copies of the pinned-chunk pipeline: streaming AVX2 stores vs memcpy, at 32 / 64 MiB chunks
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r02j; mkdir -p $O
for R in 1 2; do
  for NT in 0 1; do
    echo "nt=$NT round=$R" >> $O/host_copy_ab.jsonl
    DDL_HOST_COPY_NT=$NT timeout -k 10 200 python tools/host_chunk_tune.py 1 32,64 >> $O/host_copy_ab.jsonl 2>> $O/host_copy_ab.err || exit 1
  done
done
cat $O/host_copy_ab.jsonl
