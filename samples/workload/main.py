"""Sample pod workload (see gpushare_scheduler_extender_amd/sim/workload.py): GEMM loop inside the pod's GPU share."""
import os
import sys

sys.path.insert(0, os.environ.get("GSX_HOME", "/opt/gpushare"))
from gpushare_scheduler_extender_amd.sim.workload import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
