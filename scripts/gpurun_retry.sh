#!/bin/bash
# gpurun with retries on INFRASTRUCTURE transients only (status=transient: no box / slot, backoff,
# box lost while being prepared or taken away -- nothing of the command ran, nothing charged).  Any run of the command itself is final.
#   scripts/gpurun_retry.sh OUTFILE TIMEOUT 'command'
out=$1; to=$2; cmd=$3
for a in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $out 2>&1
  if grep -q "status=transient" $out; then   # nothing ran, nothing charged
    w=$(grep -o "retry in [0-9]*s" $out | grep -o "[0-9]*" | head -1); sleep $(( ${w:-90} + 15 )); continue
  fi
  break
done
