set -o pipefail
O=gpurun_out/r04s
mkdir -p $O
for v in lib lib_i24 lib_i32; do
  for cfg in cfg2_1m_sh3_1080p_f16 cfg3_5m_sh3_4k_f16; do
    GSM_AMD_LIB=$PWD/gsm-renderer_amd/$v/libgsm_amd.so timeout -k 10 300 python -u bench.py --config $cfg --steps 30 --warmup 5 --cpu-baseline 0 --virtual-ranks 0 --inflight-steps 0 --orbit-steps 0 > $O/b_${v}_$cfg.log 2>&1 || { tail -5 $O/b_${v}_$cfg.log; exit 1; }
    tail -1 $O/b_${v}_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v $cfg fps', round(d['value'],1), 'parity', d['parity_vs_oracle'], {k: round(v*1e3,1) for k,v in d['stages_ms'].items()})"
  done
done
