#!/usr/bin/env bash
# Container entry: print the share the device plugin gave us, then run the workload inside it (extra arguments go
# to main.py).  GSX_APP_DIR: where main.py is (the image: /app).
P=${GSX_ENV_PREFIX:-SHARED_GPU_MEM}
DEV_VAR=${P}_DEV; CON_VAR=${P}_CONTAINER
APP=${GSX_APP_DIR:-$(cd "$(dirname "$0")" && pwd)}
echo ${DEV_VAR}=${!DEV_VAR}
echo ${CON_VAR}=${!CON_VAR}
echo HIP_VISIBLE_DEVICES=$HIP_VISIBLE_DEVICES HSA_CU_MASK=${HSA_CU_MASK:-none}
exec python3 "$APP/main.py" --total="${!DEV_VAR:-0}" --allocated="${!CON_VAR:-0}" "$@"
