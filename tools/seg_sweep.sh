#!/bin/bash
for S in 2048 1984 2112 2240 1856 1536 2560; do
  echo "S=$S"; RCDC_SEG_BYTES=$S timeout -k 10 120 python tools/variants.py 41 | grep -E "scan median|parity"
done
