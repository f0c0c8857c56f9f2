# Run a command under rocprofv3 with ONE HSA runtime in the process (copy trace).
#
# rocprofv3 preloads its SDK, whose libhsa-amd-aqlprofile64 NEEDs libhsa-runtime64.so.1 and so
# loads /opt/rocm's (7.2) runtime at startup; torch's bundled HIP (7.0) then asks for
# "libhsa-runtime64.so" by its RPATH and loads torch's own copy beside it.  The app's copies run on
# torch's runtime while the SDK waits for their completion signals through the other one: it times
# out after 30 s ("completion callbacks were not delivered", no copy records, even for torch alone)
# or, when the app has released the signals' pages, faults in __cxa_finalize (rc 139).
#
# Here a directory on LD_LIBRARY_PATH (searched before aqlprofile's RUNPATH) offers torch's runtime
# under the soname the SDK asks for; torch's later RPATH load of the same file is the same inode,
# which the dynamic loader maps once.  Usage: bash tools/rocprof_one_hsa.sh <rocprofv3 args> -- <cmd>
set -e
D=${TMPDIR:-/tmp}/tk_one_hsa
mkdir -p "$D"
T=$(python3 -c "import os, torch; print(os.path.join(os.path.dirname(torch.__file__), 'lib', 'libhsa-runtime64.so'))")
ln -sf "$T" "$D/libhsa-runtime64.so.1"
export LD_LIBRARY_PATH="$D${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH}"
exec rocprofv3 "$@"
