#!/bin/bash
# Round-3 evidence at the final bench layout: tests + smoke, the config-2 bench with its
# kernel trace / PMC traffic / SQ counter passes (tools/gpu_r03.sh steps), in one session
set -o pipefail
bash tools/gpu_r03.sh test && bash tools/gpu_r03.sh bench && bash tools/gpu_r03.sh prof && bash tools/gpu_r03.sh detail
