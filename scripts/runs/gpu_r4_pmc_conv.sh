#!/bin/bash
# Round 4: PMC of the 28x28 3x3 128->128 forward conv, dma1 (default) vs the single-stage v1
set -o pipefail
bash scripts/pmc_conv.sh pmc_conv_dma1 256 28 128 128 3 2 && bash scripts/pmc_conv.sh pmc_conv_v1 256 28 128 128 3 1
