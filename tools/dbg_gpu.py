import sys, os
sys.path[:0]=['genome-weaver-align_amd','oracle','tools','tests/hostcore']
import gwa, oracle as O, synth, numpy as np
codes,names,lengths=synth.genome([("chr1",60000),("chr2",40000)],1)
seqs,rn=synth.reads(codes,lengths,500,100,2)
strs=synth.to_strings(seqs)
reads=[(rn[i],strs[i],"I"*100) for i in range(len(strs))]
gi=gwa.FMIndexOnGenome.buildFromCodes(codes,names,lengths,device=0)
os.environ["GWA_TRACE_READ"]="20"; os.environ["GWA_QTRACE_READ"]="20"; os.environ["GWA_TRACE_FILE"]="gpurun_out/gpu_trace.bin"
b=gwa.Batch(gi,gwa.AlignmentConfig(k=2.0),reads); b.run()
c=b.read_counters()
np.save('gpurun_out/gpu_counters.npy', c)
sam,off=b.results()
open('gpurun_out/gpu.sam','w').write(sam)
print("done")
