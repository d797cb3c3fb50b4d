#!/bin/bash
set -u
mkdir -p gpurun_out/dp2
export TMPDIR=/tmp
timeout -k 10 120 python tools/deferred_probe2.py 777 > gpurun_out/dp2/probe.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/dp2/probe.log | tail -60
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 200 python tools/host_micro.py balance 32768 > gpurun_out/dp2/host_micro.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/dp2/host_micro.log | tail -12
timeout -k 10 200 python tools/host_profile.py balance 32768 > gpurun_out/dp2/host_profile.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/dp2/host_profile.log | head -60
