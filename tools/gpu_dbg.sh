for v in "" "SRHIP_JIT_MANUAL_OFF=exp" "SRHIP_JIT_MANUAL_OFF=trig" "SRHIP_JIT_MANUAL_OFF=div"; do
  echo "== [$v]"; env $v timeout -k 10 200 python -u tools/debug_row.py 1000 347800 347900 2>&1 | grep -E "rows where|differs" | head -5
done
