#!/bin/bash
# passes M (dW kernel) and N (attention packed softmax) in one call
set -e
bash scripts/r3_gpu_n.sh
bash scripts/r3_gpu_m.sh
