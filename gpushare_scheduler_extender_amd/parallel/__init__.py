"""Concurrency lives in the native engine, not here: the extender's epoll loops and bind pool
(``native/engine/server.cc``), its pod / node reflectors (``informer.cc``, ``controller.cc``), the device
plugin's serving thread (``bindings.cc: PyDpServer``) and the compiled stand-ins.  The scale-out plan of the
benchmark's processes over CPUs is :mod:`gpushare_scheduler_extender_amd.utils.cpuset`."""
