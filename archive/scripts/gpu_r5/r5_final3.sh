#!/bin/bash
# round 5 final evidence pass 3 (tree with the SwiGLU-backward epilogue): same steps as pass 2
FINAL_OUT=r5_final3 exec bash scripts/gpu/r5_final2.sh
