#!/bin/bash
for g in 10 20 30 45 60 90 120; do echo "groups=$g"; python scripts/kbench.py --reps 3 --groups $g --only wgrad16,wgrad1_mode0,wgrad1_mode1; done
