# MI355X risk platform — build / test / bench / ops entry points.
# GPU targets go through gpurun (one MI355X box per call) unless run directly on a GPU host.

PY        ?= python
GPURUN    ?= /usr/local/graft/bin/gpurun
GPUS      ?= 1
STEPS     ?= 300
WARMUP    ?= 30
CONFIG    ?= cfg3

.PHONY: all build build-sanitize test-sanitize test test-gpu test-dist lint bench bench-all profile serve serve-spmd \
        wallet bonus-validate models api-test health clean help

all: build

build: ## compile the C++ runtime (_native) and the gfx950 HIP kernels (_hipk) in-tree
	$(PY) -m igaming_platform_amd._build

build-sanitize: ## host runtime with ASan/UBSan (GPU sanitizers are not available on the pool)
	$(PY) -m igaming_platform_amd._build --sanitize

test-sanitize: build ## native / engine / API tests against the ASan+UBSan host runtime (child interpreter)
	$(PY) -m pytest tests/test_sanitize.py -q

test: build ## CPU suite (golden, native runtime, engine, API, clients, gloo multi-process)
	$(PY) -m pytest tests -q -m "not gpu"

test-dist: build ## multi-process SPMD serving over gloo (world 2 and 3)
	$(PY) -m pytest tests/test_dist.py -q

test-gpu: build ## GPU suite on an MI355X (kernels vs golden / CPU executor, engine parity)
	$(GPURUN) --timeout 900 -- 'timeout -k 10 800 $(PY) -m pytest tests -q -m gpu'

lint: ## style + static checks (no third-party linters in the image)
	$(PY) tools/lint.py

bench: build ## headline: fraud scores/s + p99 on $(GPUS) GPU(s)
	$(PY) bench.py --gpus $(GPUS) --steps $(STEPS) --warmup $(WARMUP) --config $(CONFIG)

bench-all: build ## all five BASELINE configs (cfg1 CPU gRPC, cfg2-cfg5 GPU)
	$(PY) tools/bench_cfg1.py
	for c in cfg2 cfg3 cfg4 cfg5; do $(PY) bench.py --config $$c --steps 100 --warmup 10; done

profile: build ## rocprofv3 kernel trace + stats of the headline step (writes gpurun_out/prof)
	cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $(CURDIR)/gpurun_out/prof -- \
	    $(PY) $(CURDIR)/bench.py --steps 50 --warmup 10

serve: build ## risk service (gRPC :9082, HTTP :8082)
	$(PY) -m igaming_platform_amd.serve

serve-spmd: build ## one process per GPU; rank 0 serves the API
	$(PY) -m torch.distributed.run --nnodes=1 --nproc-per-node $(GPUS) --master-addr 127.0.0.1 \
	    -m igaming_platform_amd.serve --backend gpu

wallet: ## wallet service (gRPC :9080) against RISK_SERVICE_URL
	$(PY) -m igaming_platform_amd.wallet.serve

bonus-validate: ## validate the bonus rule DSL file (CONFIG_PATH)
	$(PY) -m igaming_platform_amd.bonus validate

models: ## write the synthetic random-init ONNX models of the five configs to models/
	$(PY) tools/gen_models.py --out models

api-test: ## score one transaction against a running risk service
	$(PY) -c "from igaming_platform_amd.clients.risk_client import RiskClient as C; \
	print(C('127.0.0.1:9082').score('demo-account', 150000, 'deposit', device_id='d1'))"

health: ## gRPC + HTTP health of a running risk service
	$(PY) -c "from igaming_platform_amd.clients.risk_client import RiskClient as C; print(C('127.0.0.1:9082').health())"
	curl -fsS http://127.0.0.1:8082/ready && echo

clean:
	rm -rf build igaming_platform_amd/*.so gpurun_out/prof .pytest_cache

help:
	@grep -E '^[a-zA-Z_-]+:.*?## ' $(MAKEFILE_LIST) | awk 'BEGIN {FS = ":.*?## "}; {printf "%-16s %s\n", $$1, $$2}'
