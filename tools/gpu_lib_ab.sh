# A/B of two in-tree builds of libgsm_amd (LIBS="lib lib_x"): the GPU parity tests on the first, then
# bench lines of configs 2 and 3 for each (static + orbit), alternating builds twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-libab}
mkdir -p $O
L1=$(echo ${LIBS:-lib} | cut -d' ' -f1)
GSM_AMD_LIB=$PWD/gsm-renderer_amd/$L1/libgsm_amd.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_depthfirst.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log | cut -c1-300; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for v in ${LIBS:-lib}; do
  for cfg in cfg2_1m_sh3_1080p_f16 cfg3_5m_sh3_4k_f16; do
    GSM_AMD_LIB=$PWD/gsm-renderer_amd/$v/libgsm_amd.so timeout -k 10 300 python -u bench.py --config $cfg --steps 50 --warmup 5 --cpu-baseline 0 --virtual-ranks 0 --inflight-steps 0 > $O/b_${v}_${cfg}_$rep.log 2>&1 || { tail -5 $O/b_${v}_${cfg}_$rep.log; exit 1; }
    tail -1 $O/b_${v}_${cfg}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); o=d.get('orbit') or {}; print('$v $cfg fps', round(d['value'],1), 'parity', d['parity_vs_oracle'], 'orbit', round(o.get('value',0),1), 'oblend', round(o.get('blend_ms',0)*1e3,1), 'blend', round(d['stages_ms']['blend']*1e3,1), 'proj', round(d['stages_ms']['project']*1e3,1))"
  done
done
done
