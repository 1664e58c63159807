"""Development harness around the product package (not shipped in it): the Python kubelet stand-in
(:mod:`.agent`), the in-process cluster launcher (:mod:`.cluster`), the BASELINE configurations
(:mod:`.configs`), the scale and isolation benchmarks (:mod:`.scale`, :mod:`.isolation`) and the sample pod
workload (:mod:`.workload`, the ``samples/workload`` container's entry point)."""
