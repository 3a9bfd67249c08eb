# Convenience targets (plain make; all native work goes through ddl_amd/_build.py).
PY ?= python

.PHONY: build test test-gpu bench resources clean
build:
	$(PY) -m ddl_amd._build

test: build
	$(PY) -m pytest tests -x -q -m "not gpu"

test-gpu: build
	$(PY) -m pytest tests -x -q -m gpu

bench: build
	$(PY) bench.py

resources:
	$(PY) tools/kernel_resources.py > profiles/kernel_resources_gfx950.txt

clean:
	rm -rf build ddl_amd/*.so
