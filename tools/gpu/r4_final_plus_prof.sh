#!/bin/bash
# closing check (full GPU tier, smoke, bench, GPT-2, attention) and then the step profile
set -o pipefail
bash tools/gpu/r4_final_check.sh || exit $?
bash tools/gpu/r4_prof_now.sh
