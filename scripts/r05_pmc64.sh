#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one each, MI355X_MICROARCH.md's HBM recipe) of the
# headline step kernel in float64 (step_kernel<double, ...>, the fp64 leg) and, for
# comparison in the same box, float32; calibrated on qs_calib_copy.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-p64}
for prec in 8 4; do
  for c in FETCH_SIZE WRITE_SIZE; do
    PMC_PRECISION=$prec timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/${TAG}_${prec}_$c -o run \
      --output-format csv -- python3 scripts/pmc_probe.py > gpurun_out/${TAG}_${prec}_$c.log 2>&1
    rc=$?; echo "pmc $prec $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  bytes=$(python3 -c "import bench; print(bench.bytes_per_agent_step('one_d_pid', 'multihover', 8, precision=$prec))")
  python3 scripts/pmc_report.py gpurun_out/${TAG}_${prec}_FETCH_SIZE gpurun_out/${TAG}_${prec}_WRITE_SIZE $((1 << 28)) 131072 \
    $bytes 16384 8 one_d_pid $prec > gpurun_out/${TAG}_pmc_traffic_$prec.json && cat gpurun_out/${TAG}_pmc_traffic_$prec.json
  rm -rf gpurun_out/${TAG}_${prec}_FETCH_SIZE gpurun_out/${TAG}_${prec}_WRITE_SIZE
done
