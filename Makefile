# Build / test / benchmark entry points (CI: .github/workflows/ci.yml).
PY ?= python3
.PHONY: build test test-gpu sanitize bench configs clean
build: ; $(PY) native/build.py
test: build ; $(PY) -m pytest tests -m "not gpu" -q
test-gpu: build ; $(PY) -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
sanitize: ; $(PY) native/build.py asan tsan
bench: build ; $(PY) bench.py
configs: build ; $(PY) -m gsxtools.configs
clean: ; rm -rf build gpushare_scheduler_extender_amd/_native/*.so gpushare_scheduler_extender_amd/_native/gsx-*
