# C3 at the driver's step counts per pipeline shape (front x back streams),
# alternating, two reps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && mkdir -p gpurun_out/sab
for rep in 1 2; do
  for cfg in "1 3" "1 2" "1 4" "2 3" "2 4"; do
    set -- $cfg
    timeout -k 10 200 python bench.py --front-streams $1 --back-streams $2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/sab/f$1b$2.$rep.json 2> gpurun_out/sab/f$1b$2.$rep.err || { tail -5 gpurun_out/sab/f$1b$2.$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/sab/f$1b$2.$rep.json')); print('front $1 back $2 rep $rep', round(d['value']/1e6,3), 'M', d['roofline']['frac'])"
  done
done
