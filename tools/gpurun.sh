#!/bin/bash
# Rebuild everything in-tree on the CPU, then run a command on a GPU box.
# usage: tools/gpurun.sh TIMEOUT 'command'
set -e
cd "$(dirname "$0")/.."
make -s -C tmlibrary_amd/csrc -j8
make -s -C tools/mb
exec timeout $(( $1 + 900 )) /usr/local/graft/bin/gpurun --timeout "$1" -- "$2"
