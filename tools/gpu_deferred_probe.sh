#!/bin/bash
set -u
mkdir -p gpurun_out/dp
timeout -k 10 120 python tools/deferred_probe.py 777 > gpurun_out/dp/probe.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/dp/probe.log | tail -25; exit $rc
