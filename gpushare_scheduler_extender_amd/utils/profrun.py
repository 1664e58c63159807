"""Run a module under cProfile and dump the stats on exit (also on SIGTERM).

    python -m gpushare_scheduler_extender_amd.utils.profrun OUT.prof some.module [args...]

The process harness (``gsxtools/cluster.py``) wraps its children with this when
``GSX_CPROFILE_DIR`` is set, to see where the control plane spends its CPU.
"""
import cProfile
import runpy
import signal
import sys


def main():
    out, mod = sys.argv[1], sys.argv[2]
    sys.argv = [mod] + sys.argv[3:]

    def _term(*_):
        raise KeyboardInterrupt

    signal.signal(signal.SIGTERM, _term)
    pr = cProfile.Profile()
    pr.enable()
    try:
        runpy.run_module(mod, run_name="__main__", alter_sys=True)
    except (KeyboardInterrupt, SystemExit):
        pass
    finally:
        pr.disable()
        pr.dump_stats(out)


if __name__ == "__main__":
    main()
