#!/bin/bash
set -e
bash scripts/r3_gpu_x.sh
bash scripts/r3_gpu_w.sh
bash scripts/r3_gpu_v.sh
