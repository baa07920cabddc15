#!/bin/bash
# round 5 final evidence pass 4 (tree with the fused clip norm, ZeRO-1 config-3 variant, adapter-copy
# transpose path): same steps as pass 2
FINAL_OUT=r5_final4 exec bash scripts/gpu/r5_final2.sh
