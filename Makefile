# Convenience targets (the reference's makefile alembic targets map to `python -m smsgate_amd db ...`).
PY ?= python
.PHONY: build test test-gpu bench upgrade downgrade current history stamp smoke

build:            ## compile the HIP kernels for gfx950
	$(PY) -m smsgate_amd.ops.build --force
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
