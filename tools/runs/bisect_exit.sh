cd $GRAFT_REPO_ROOT
run() { timeout -k 5 120 python -c "$2" > gpurun_out/bisect_$1.log 2>&1; echo "$1 rc=$?" >> gpurun_out/bisect.txt; }
mkdir -p gpurun_out; : > gpurun_out/bisect.txt
run host "import torch,numpy as np; import vds_amd as v; v.chunk.encode_host(16,list(range(20)),np.zeros(1000,np.uint8)); print('ok')"
run hostnotorch "import numpy as np; import vds_amd as v; v.chunk.encode_host(16,list(range(20)),np.zeros(1000,np.uint8)); print('ok')"
run restorehost "import torch,numpy as np; import vds_amd as v; c=v.chunk.encode_host(4,[1,2,3,4],np.zeros(100,np.uint8)); v.ChunkRestore(4,[1,2,3,4]).restore(c); print('ok')"
run batch "import torch,numpy as np; import vds_amd as v; v.encode_host_batch(16,list(range(20)),[np.zeros(1000,np.uint8)]*3); print('ok')"
run batchnotorch "import numpy as np; import vds_amd as v; v.encode_host_batch(16,list(range(20)),[np.zeros(1000,np.uint8)]*3); print('ok')"
run device "import torch; import vds_amd as v; t=torch.zeros(1000,dtype=torch.uint8,device='cuda'); o=torch.zeros((20,600),dtype=torch.uint8,device='cuda'); v.encode_device(16,list(range(20)),t,1000,1000,1,[o[i].data_ptr() for i in range(20)],600); torch.cuda.synchronize(); print('ok')"
run restoredev "import torch; import vds_amd as v; t=torch.zeros(1000,dtype=torch.uint8,device='cuda'); o=torch.zeros((20,600),dtype=torch.uint8,device='cuda'); v.encode_device(16,list(range(20)),t,1000,1000,1,[o[i].data_ptr() for i in range(20)],600); r=torch.zeros(1000,dtype=torch.uint8,device='cuda'); v.restore_device(16,list(range(4,20)),[o[i].data_ptr() for i in range(4,20)],34,0,1000%32,1,r,0); torch.cuda.synchronize(); print('ok')"
cat gpurun_out/bisect.txt
