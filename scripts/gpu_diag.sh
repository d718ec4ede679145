cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
(timeout 120 python scripts/diag_hip.py plain; timeout 120 python scripts/diag_hip.py torch_first; echo HIP_VISIBLE=$HIP_VISIBLE_DEVICES ROCR=$ROCR_VISIBLE_DEVICES; ls -la /dev/kfd /dev/dri | head) > gpurun_out/diag.log 2>&1
