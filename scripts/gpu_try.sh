#!/bin/bash
# Run one gpurun call; when gpurun reports no box / an infrastructure hiccup (exit 3: nothing ran,
# nothing charged) wait and ask again, up to 6 times.  Any other exit code is returned as is.
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun "$@"
  rc=$?
  if [ $rc -ne 3 ]; then exit $rc; fi
  sleep 45
done
exit 3
