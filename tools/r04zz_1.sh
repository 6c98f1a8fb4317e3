#!/bin/bash
# Round 4 final tree, C3 (1280x720/2000): kernel stats + FETCH/WRITE + calibration, then read-request sizes + SQ counts.
set -e
bash tools/profile_round.sh r04zz a
bash tools/profile_round.sh r04zz b
