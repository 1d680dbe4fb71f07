# dev helper: submit one gpurun call, resubmitting only while the pool answers "no box / slot
# free" (exit 3: nothing ran, nothing charged).  Usage: gpurun_when_free.sh <out> <timeout> <cmd>
out=$1; to=$2; cmd=$3
for i in $(seq 1 30); do
  timeout $((to + 1500)) /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$out" 2>&1
  rc=$?
  echo "EXIT $rc" >> "$out"
  if [ $rc -ne 3 ]; then exit $rc; fi
  sleep 90
done
