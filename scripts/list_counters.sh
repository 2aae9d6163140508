#!/bin/bash
# List rocprofv3 PMC counters available on this GPU (gfx950) into gpurun_out/.
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > "$GRAFT_REPO_ROOT/gpurun_out/counters.txt" 2>&1 || rocprofv3 --list-avail > "$GRAFT_REPO_ROOT/gpurun_out/counters.txt" 2>&1
