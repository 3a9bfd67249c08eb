# Round 5, sixth box: does the zero-copy gather's rate depend on how the host source is mapped (page size)?
# The wave-granular kernel that reached 57.2 GB/s on hipHostMalloc memory fell to 174k samples/s in the loader,
# whose source is a registered POSIX shm segment (profiles/r5_zerocopy/fifth/).
source tools/gpu_job.sh
unset DDL_BACKEND
run 60 thp bash -c 'for f in enabled shmem_enabled defrag; do echo "$f: $(cat /sys/kernel/mm/transparent_hugepage/$f 2>/dev/null)"; done; grep -i huge /proc/meminfo'
for mem in hostmalloc shm anon4k anonthp; do
  run 300 zc_probe_$mem benchmarks/bin/probe_zerocopy_read 4096 5 $mem
done
