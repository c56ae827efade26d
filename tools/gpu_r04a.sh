#!/bin/bash
# Round-4 first session: C5 bucket-ends patch A/B (render GPU tests with it, then the bench's C5
# section alternating against ab/libomr_old.so), then the all-sections profile (tools/profile_r04.sh).
set -o pipefail
timeout -k 10 900 bash tools/c5_lib_ab.sh || exit $?
timeout -k 10 900 bash tools/profile_r04.sh r04a_prof || exit $?
echo R04A OK
