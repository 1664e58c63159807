"""gpushare_scheduler_extender_amd — GPU-memory sharing for Kubernetes on AMD Instinct MI355X.

A from-scratch, MI355X-native re-design of the capabilities of
bnulwh/gpushare-scheduler-extender:

* ``core``         native (C++) ledger/binpack engine + the cluster-state controller
* ``extender``     kube-scheduler extender HTTP API (filter / bind / inspect / version / pprof / metrics)
* ``k8s``          async Kubernetes REST+watch client, informers, leader election
* ``deviceplugin`` kubelet device plugin (v1beta1 gRPC) handing out /dev/kfd + /dev/dri render nodes
* ``ops``          amdsmi device library, HIP/CDNA4 kernels (CU probe, HBM touch, MFMA GEMM), CU masks
* ``models``       wire types, naming profiles, pod/node accessors, quantities
* ``parallel``     client-go-style rate-limited work queue (dedup, per-item backoff, bucket limiter)
* ``sim``          cluster harness (compiled fake apiserver / scheduler / node agent), BASELINE configs
* ``cli``          ``kubectl inspect gpushare`` equivalent
"""
__version__ = "0.1.0"
