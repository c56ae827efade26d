#!/bin/bash
# Round-3 full GPU session: every GPU test, smoke, the driver's bench command, the headline
# rocprofv3 trace + HBM traffic (tools/profile_r03.sh), the JPEG trace + SQ counters
# (tools/profile_jpeg_r03.sh).  Each step under its own time limit; the first failure ends it.
set -o pipefail
T=${1:-r03full}
bash tools/gpu_run.sh $T tests smoke bench || exit $?
timeout -k 10 600 bash tools/profile_r03.sh ${T}_prof || exit $?
timeout -k 10 600 bash tools/profile_jpeg_r03.sh ${T}_jpeg > /dev/null || exit $?
echo FULL OK
