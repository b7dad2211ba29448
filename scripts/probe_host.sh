set -x
nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"
cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /proc/self/cgroup; lscpu | head -20
env | grep -E "OMP|MAX_JOBS|HIP|ROCR|GPU" 
free -g
