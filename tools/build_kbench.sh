#!/bin/bash
# builds tools/kbench (dev microbenchmark) against the in-tree libdsocr.so
set -e
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/kbench.cpp -o tools/kbench \
  -Ldeepseek-ocr.rs_amd/lib -ldsocr -Wl,-rpath,'$ORIGIN/../deepseek-ocr.rs_amd/lib' -Wl,-rpath,/opt/rocm/lib
