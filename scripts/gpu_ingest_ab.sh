#!/bin/bash
# Ingest leg A/B on one box: bench.py (ingest leg only) on $WLS for each "ENV=... LIB" configuration
# listed in $CONFIGS (';'-separated; LIB empty = the product library).  Output: ms per ingest.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp; R=$PWD
IFS=';' read -ra CF <<< "${CONFIGS:-base}"
for round in 1 2; do
  for wl in ${WLS:-C3 T}; do
    for c in "${CF[@]}"; do
      env $( [ "$c" = base ] || echo $c ) timeout -k 10 200 python bench.py --workload $wl --no-c1 --no-cpu-baseline --no-e2e \
        --no-cdr --no-frag > gpurun_out/iab.json 2> gpurun_out/iab.err || { echo "FAIL $c"; tail -5 gpurun_out/iab.err; exit 4; }
      python3 -c "import json; d=json.loads([l for l in open('gpurun_out/iab.json') if l.startswith('{')][-1]); i=d['ingest']; print('$wl', '$c'.ljust(60), 'ingest %.1f us' % (i['ms']*1e3), 'acc', i['accepted'])"
    done
  done
done
