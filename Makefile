# Convenience targets (everything is also reachable through python -m ...).
PY ?= python3

.PHONY: build native canary test test-gpu sanitize analyze bench suite soak probes inspect run-fixture image clean

build:            ## C++ core (pybind11 .so) + gfx950 HIP canary, in-tree
	$(PY) -m k8s_gpu_device_plugin_amd._build
native:
	$(PY) -m k8s_gpu_device_plugin_amd._build --no-canary
canary:
	$(PY) -c "from k8s_gpu_device_plugin_amd import _build; _build.build_canary()"
test:             ## CPU suite (fixture backend, gloo)
	$(PY) -m pytest tests -q -m "not gpu"
test-gpu:         ## needs an MI355X (e.g. through gpurun)
	$(PY) -m pytest tests -q -m gpu
sanitize:         ## native self-test, then the integration tests, under ASan+UBSan and TSan
	$(PY) -m k8s_gpu_device_plugin_amd._build --sanitize address
	$(PY) -m k8s_gpu_device_plugin_amd._build --sanitize thread
	$(PY) -m pytest tests/test_sanitized_suite.py -q
analyze:          ## clang static analyzer over native/*.cpp (fails on any finding)
	scripts/analyze.sh
bench:
	$(PY) bench.py --gpus 1 --steps 20 --warmup 3
suite:            ## BASELINE.json configs 1-5 + scaling + health propagation
	$(PY) -m k8s_gpu_device_plugin_amd.benchmark.suite --json suite.json
soak:             ## daemon under Allocate + scrapes + /restart every 250 ms for 2 min (real backend if present)
	$(PY) scripts/soak.py --seconds 120 --restart-every 0.25
probes:           ## scrape-path, concurrency and idle-gap probes (JSON lines)
	$(PY) scripts/scrape_probe.py
	$(PY) scripts/concurrency_probe.py
	$(PY) scripts/idle_probe.py
inspect:          ## what this node would advertise, and where 2/4/8-device pods would go
	$(PY) -m k8s_gpu_device_plugin_amd --inspect
run-fixture:      ## daemon on a fake 8x CPX node, no hardware needed
	$(PY) -m k8s_gpu_device_plugin_amd --backend fixture --fixture 8gpu_cpx_nps2 --strategy single \
	  --plugin-dir /tmp/amdgpu-dp --web-listen-address 127.0.0.1:9100
image:
	docker build -f deploy/Dockerfile -t amdgpu-device-plugin:0.1.0 .
clean:
	rm -rf build k8s_gpu_device_plugin_amd/_native*.so k8s_gpu_device_plugin_amd/ops/libamdgpu_canary.so
