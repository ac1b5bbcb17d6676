#!/bin/bash
# Head bytes 48..63: loaded only for non-DATA first submessages (product) vs always (ABL_HEAD_EAGER), and the
# previous commit's parse (abl_base/rtps_rx.hip if present), T / C2 / C4, same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; mkdir -p gpurun_out build; export TMPDIR=/tmp
C=rustdds-io_uring_amd/csrc
(cd $C && /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wno-unused-function -DABL_HEAD_EAGER -shared \
   -o $R/build/librtps_eager.so rtps_rx.hip rtps_cdr.hip rtps_frag.hip rtps_ingest.hip rtps_udp.cpp rtps_pump.cpp) || exit 2
libs="$C/../librtps_rx.so build/librtps_eager.so"
if [ -f abl_base/rtps_rx.hip ]; then
  cp $C/*.h abl_base/ && (cd abl_base && /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC \
    -Wno-unused-function -shared -o $R/build/librtps_base.so rtps_rx.hip $R/$C/rtps_cdr.hip $R/$C/rtps_frag.hip \
    $R/$C/rtps_ingest.hip $R/$C/rtps_udp.cpp $R/$C/rtps_pump.cpp -I$R/$C) || exit 2
  libs="$libs build/librtps_base.so"
fi
for rep in 1 2; do
for lib in $libs; do
  for wl in T C2 C4; do
    RTPS_RX_LIB=$R/$lib timeout -k 10 200 python bench.py --workload $wl --steps 40 --no-cpu-baseline --no-e2e \
      --no-cdr --no-frag --no-ingest --no-c1 > gpurun_out/head_abl.log 2>&1 || { tail -5 gpurun_out/head_abl.log; exit 4; }
    python -c "import json; d=json.loads(open('gpurun_out/head_abl.log').read().strip().splitlines()[-1]); print('$lib', '$wl', 'kernel %.1f us' % (d['roofline']['kernel_ms']*1e3))"
  done
done
done
