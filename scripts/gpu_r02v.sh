#!/bin/bash
# SQ instruction-mix / stall counters of the current gossip round (two PMC passes)
bash scripts/pmc_sq.sh r02v --workload gossip --no-vivaldi
