#!/bin/bash
# queue a gpurun call: retry ONLY while the pool has no free box (rc 3, nothing ran, nothing charged)
CMD="$1"; OUT="$2"; TMO="${3:-1200}"
for i in $(seq 1 20); do
  timeout $((TMO + 1800)) /usr/local/graft/bin/gpurun --timeout $TMO -- "$CMD" > "$OUT" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -qE "no free box right now|slot\(s\) on this pod are busy" "$OUT"; then echo "rc=$rc" >> "$OUT"; exit $rc; fi
  sleep 150
done
