# C5 (int8) today: the pipelined line, then a serial kernel trace with
# per-kernel stats (which passes the int8 step spends its time in).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && mkdir -p gpurun_out/c5p && export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload c5 --steps 60 --warmup 10 --no-cpu-baseline > gpurun_out/c5p/bench.json 2> gpurun_out/c5p/bench.err || { tail -5 gpurun_out/c5p/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/c5p/bench.json')); print('C5', d['value'], d['roofline']['frac'], d['roofline'].get('achieved'), d.get('stages'))"
rm -rf gpurun_out/c5p/run
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5p/run -o run -- \
    python3 bench.py --workload c5 --serial --steps 20 --warmup 5 --no-cpu-baseline --no-profile > gpurun_out/c5p/serial.log 2>&1 || { tail -5 gpurun_out/c5p/serial.log; exit 1; }
python3 tools/trace_summary.py $(find gpurun_out/c5p/run -name '*kernel_trace.csv' | head -1) "C5 serial" > gpurun_out/c5p/summary.txt
head -30 gpurun_out/c5p/summary.txt
