# r4b: graphed-schedule contention knobs + lab small-token study, then DiffuSeq-XL HBM headroom.
bash tools/gpu/graph_ab3.sh && bash tools/gpu/xl_mem.sh
