# Convenience targets (the reference's makefile alembic targets map to `python -m smsgate_amd db ...`).
PY ?= python
.PHONY: build native sanitize test test-gpu bench bus-bench upgrade downgrade current history stamp smoke

build: native     ## compile the HIP kernels for gfx950 (+ the native broker)
	$(PY) -m smsgate_amd.ops.build --force
native:           ## C++ broker smsgate-busd (+ its ASan/UBSan build)
	$(PY) -m smsgate_amd.native.build --force --sanitize
bus-bench:        ## Python vs native broker throughput
	$(PY) scripts/bus_bench.py
test:             ## CPU test suite
	$(PY) -m pytest tests -x -q -m "not gpu"
test-gpu:         ## GPU tests (MI355X)
	$(PY) -m pytest tests -x -q -m gpu
bench:            ## headline benchmark, one GPU
	$(PY) bench.py
smoke:
	$(PY) __graft_entry__.py smoke
upgrade:
	$(PY) -m smsgate_amd db upgrade
downgrade:
	$(PY) -m smsgate_amd db downgrade
current:
	$(PY) -m smsgate_amd db current
history:
	$(PY) -m smsgate_amd db history
stamp:
	$(PY) -m smsgate_amd db stamp
