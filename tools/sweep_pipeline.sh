#!/bin/bash
# Pipeline depth / intersect grid share / node hand-over re-sweep after the 5-waves-per-SIMD k_trace build
# (the shading now shares the traversal's CUs, so the round-2 optimum may have moved).
exec bash tools/sweep_cfg.sh \
  "base|--pipeline 8" \
  "p10|--pipeline 10" \
  "p12|--pipeline 12" \
  "p8g30|--pipeline 8 --tune trace_grid_frac=0.3" \
  "p8g22|--pipeline 8 --tune trace_grid_frac=0.22" \
  "p10g25|--pipeline 10 --tune trace_grid_frac=0.25" \
  "p12g22|--pipeline 12 --tune trace_grid_frac=0.22" \
  "ew16|--pipeline 8 --tune early_walk=16" \
  "ew32|--pipeline 8 --tune early_walk=32" \
  "base2|--pipeline 8"
