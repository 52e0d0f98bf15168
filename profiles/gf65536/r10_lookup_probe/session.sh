set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r7d; mkdir -p $O /tmp/bp
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -o /tmp/bp/bperm_probe scripts/bperm_probe.hip > $O/build.log 2>&1 &&
timeout -k 10 60 /tmp/bp/bperm_probe > $O/bperm.json 2>&1; rc=$?; cat $O/bperm.json; exit $rc
