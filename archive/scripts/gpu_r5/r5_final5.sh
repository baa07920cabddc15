#!/bin/bash
# round 5 final evidence pass 5 (final tree: clip-norm partials from every dW GEMM): same steps as pass 2
FINAL_OUT=r5_final5 exec bash scripts/gpu/r5_final2.sh
