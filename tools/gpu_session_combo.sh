#!/bin/bash
# The drop-in session (its tests and A/B), then the round's measurement session.  usage: TAG
set -o pipefail
bash tools/gpu_session_dropin.sh $1_d || exit 1
bash tools/gpu_session_final_r4.sh $1 || exit 1
