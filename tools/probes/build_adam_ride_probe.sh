#!/bin/bash
# Builds tools/probes/adam_ride_probe (default flags, the compiler packs the float4 Adam into v_pk_*) and
# adam_ride_probe_nopk (-fno-slp-vectorize: no packed fp32 in the Adam body), plus their ISA listings.
set -e
cd "$(dirname "$0")"
C=../../distributed-continuous-training-with-airflow-pytorch-distributed-ddp-_amd/csrc
F="--offload-arch=gfx950 -O3 -std=c++17 -I$C -I/opt/rocm/include -Wno-unused-result -Wno-unused-variable"
/opt/rocm/bin/hipcc $F -x hip adam_ride_probe.hip $C/knobs.cpp -o adam_ride_probe
/opt/rocm/bin/hipcc $F -fno-slp-vectorize -x hip adam_ride_probe.hip $C/knobs.cpp -o adam_ride_probe_nopk
