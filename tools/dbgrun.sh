cp orion-kmer_amd/build_dbg/liborion_kmer.so orion-kmer_amd/build/liborion_kmer.so
OKM_DEBUG_SYNC=1 timeout -k 5 45 python tools/debug_count.py tiny > gpurun_out/dbg.log 2>&1
