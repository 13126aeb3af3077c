# Otedama (MI355X) — build, test, bench, profile.
# Parity with the reference Makefile targets (build/test/test-unit/bench/fuzz/lint/docker/release);
# the toolchain is ROCm (hipcc for gfx950) + g++ + Python instead of Go.

PYTHON      ?= python3
JOBS        ?= 8
GPURUN      ?= /usr/local/graft/bin/gpurun
IMAGE       ?= otedama-mi355x
VERSION     := $(shell $(PYTHON) -c "from otedama_amd.version import VERSION; print(VERSION)" 2>/dev/null)

export PYTHONPATH := $(CURDIR)$(if $(PYTHONPATH),:$(PYTHONPATH))

.PHONY: help build rebuild test test-unit test-gpu test-multiproc bench bench-cpu profile fuzz lint docs \
        docker-build docker-run release-check clean smoke doctor sanitize

help: ## Display this help message
	@grep -E '^[a-zA-Z_-]+:.*?## ' $(MAKEFILE_LIST) | awk 'BEGIN {FS = ":.*?## "}; {printf "  %-16s %s\n", $$1, $$2}'

build: ## Compile the gfx950 HIP kernels + C++ runtime into otedama_amd/_native*.so (incremental)
	$(PYTHON) -m otedama_amd._build -j $(JOBS)

rebuild: ## Force a full native rebuild
	$(PYTHON) -m otedama_amd._build -j $(JOBS) --force

test: build ## Run the CPU test suite (what CI runs; GPU tests are skipped without a GPU)
	$(PYTHON) -m pytest tests -x -q -m "not gpu"

test-unit: build ## Fast unit tests (no sockets / subprocesses)
	$(PYTHON) -m pytest tests -x -q -m "not gpu" -k "not integration and not multiproc and not node"

test-multiproc: build ## Multi-process node tests over gloo (world_size 2)
	$(PYTHON) -m pytest tests/test_node_multiproc.py -x -q

test-gpu: build ## GPU tests + bench on a real MI355X through gpurun
	$(GPURUN) --timeout 900 -- 'bash tools/gpu_bench.sh'

bench: build ## Headline benchmark (1 GPU; use torchrun for N>1, see README)
	$(PYTHON) bench.py

bench-cpu: build ## Reference-style single-thread CPU SHA-256d benchmark
	$(PYTHON) -m otedama_amd bench --device cpu --threads 1

profile: build ## rocprofv3 kernel trace + SQ counters (writes gpurun_out/prof*)
	$(GPURUN) --timeout 900 -- 'bash tools/gpu_prof.sh'

fuzz: ## Property/fuzz tests for the SV2 frame codec and message decoders
	$(PYTHON) -m pytest tests -q -k "fuzz or frame"

sanitize: ## Host-only TSan + ASan/UBSan builds of the C++ runtime + job-epoch race stress
	bash tools/sanitize/run.sh 4

lint: ## Byte-compile everything (no third-party linters in the image)
	$(PYTHON) -m compileall -q otedama_amd tests bench.py __graft_entry__.py

smoke: build ## One tiny SHA-256d + scrypt search on cuda:0
	$(PYTHON) -c "import __graft_entry__ as g; g.smoke()"

doctor: ## Run the self-diagnostic checks
	$(PYTHON) -m otedama_amd doctor

docs: ## Regenerate docs/METRICS.md from the engine + pool metric registries
	$(PYTHON) tools/gen_metrics_doc.py > docs/METRICS.md

docker-build: ## Build the ROCm runtime image
	docker build --build-arg VERSION=$(VERSION) -t $(IMAGE):$(VERSION) .

docker-run: ## Run the miner in Docker with the GPUs passed through
	docker run --rm -it --device=/dev/kfd --device=/dev/dri --group-add video \
		-e HSA_ENABLE_IPC_MODE_LEGACY=0 $(IMAGE):$(VERSION) run --no-tui

release-check: lint test ## Verify readiness for release
	@echo "release-check OK for $(VERSION)"

clean: ## Remove build artefacts
	rm -rf build otedama_amd/_native*.so .pytest_cache
	find . -name __pycache__ -type d -prune -exec rm -rf {} +
