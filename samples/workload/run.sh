#!/usr/bin/env bash
# Container entry: print the share the device plugin gave us, then run the workload inside it.
P=${GSX_ENV_PREFIX:-SHARED_GPU_MEM}
DEV_VAR=${P}_DEV; CON_VAR=${P}_CONTAINER
echo ${DEV_VAR}=${!DEV_VAR}
echo ${CON_VAR}=${!CON_VAR}
echo HIP_VISIBLE_DEVICES=$HIP_VISIBLE_DEVICES HSA_CU_MASK=${HSA_CU_MASK:-none}
exec python3 /app/main.py --total="${!DEV_VAR}" --allocated="${!CON_VAR}"
