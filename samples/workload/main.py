"""Sample pod workload (see gsxtools/workload.py): GEMM loop inside the pod's GPU share."""
import os
import sys

sys.path.insert(0, os.environ.get("GSX_HOME", "/opt/gpushare"))
from gsxtools.workload import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
