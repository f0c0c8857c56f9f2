set -o pipefail
# r02d: isolated layer times with reused vs rotated (fresh) output buffers; per-kernel
# durations of the network's compute-only step (rocprof kernel trace)
mkdir -p gpurun_out/r02d
timeout -k 10 300 python -u tools/bench_block.py '[{}]' "" 1 > gpurun_out/r02d/block_rot1.txt 2>&1 &&
timeout -k 10 300 python -u tools/bench_block.py '[{}]' "" 6 > gpurun_out/r02d/block_rot6.txt 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r02d/net -o run -- python3 bench.py --steps 3 --warmup 1 --skip-cpu --no-trace > gpurun_out/r02d/net.log 2>&1
