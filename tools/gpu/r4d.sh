# r4d: DiffuSeq-XL HBM headroom, then PMC passes on the L = 128 attention kernels.
bash tools/gpu/xl_mem.sh && bash tools/gpu/pmc_a128.sh
