#!/bin/bash
# gemm8 + SAB microbenchmarks on the GPU box (one gpurun call). A step that fails its checks goes on
# to the next; a crash / fault / timeout (rc 124, 134, 137, 139) ends the call.
set -o pipefail
OUT=gpurun_out/${1:-g8b}
mkdir -p $OUT
step() { local name=$1; shift; timeout -k 10 200 "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "[$name rc=$rc]"; tail -${TAILN:-40} $OUT/$name.log;
         case $rc in 124|134|137|139) exit $rc ;; esac; }
step g8bench ./tools/g8bench 20
TAILN=12 step g8abl ./tools/g8abl 10 abl
TAILN=4 step sab_w4 ./tools/sabbench 10 0 4
TAILN=4 step sab_w8 ./tools/sabbench 10 0 8
TAILN=4 step sab_s8 ./tools/sabbench 10 8 4
exit 0
