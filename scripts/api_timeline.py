# HIP API + kernel timeline of one call window from a rocprofv3 --hip-runtime-trace --kernel-trace directory:
#   python scripts/api_timeline.py DIR KERNEL_SUBSTRING CALLS_BEFORE  (the window opens CALLS_BEFORE calls before
#   the third-last launch of the kernel and closes before the second-last)
import csv,sys
d=sys.argv[1]
api=list(csv.DictReader(open(d+'/run_hip_api_trace.csv')))
ks={int(r['Correlation_Id']):r for r in csv.DictReader(open(d+'/run_kernel_trace.csv'))}
cs={}
try:
    for r in csv.DictReader(open(d+'/run_memory_copy_trace.csv')): cs[int(r['Correlation_Id'])]=r
except Exception: pass
api=[a for a in api if a['Function'] not in ('hipGetLastError','hipGetDevice','hipSetDevice','hipDeviceGetAttribute','hipGetDeviceCount','hipCtxGetCurrent','hipDevicePrimaryCtxGetState','hipStreamIsCapturing','hipGetDevicePropertiesR0600','hipPointerGetAttributes')]
# find the compute syncs: pick a window in the middle: find indices of 'validate_pack_kernel' launches
idx=[i for i,a in enumerate(api) if int(a['Correlation_Id']) in ks and sys.argv[2] in ks[int(a['Correlation_Id'])]['Kernel_Name']]
i0=idx[-3]-int(sys.argv[3]); i1=idx[-2]-int(sys.argv[3])
t0=int(api[i0]['Start_Timestamp'])
for a in api[i0:i1]:
    c=int(a['Correlation_Id']); s=(int(a['Start_Timestamp'])-t0)/1e3; du=(int(a['End_Timestamp'])-int(a['Start_Timestamp']))/1e3
    x=''
    if c in ks:
        k=ks[c]; x=' -> %s gpu %.1f-%.1f'%(k['Kernel_Name'].replace('accord::(anonymous namespace)::','').split('(')[0][:40],(int(k['Start_Timestamp'])-t0)/1e3,(int(k['End_Timestamp'])-t0)/1e3)
    elif c in cs:
        k=cs[c]; x=' -> copy %s gpu %.1f-%.1f'%(k.get('Direction',''),(int(k['Start_Timestamp'])-t0)/1e3,(int(k['End_Timestamp'])-t0)/1e3)
    print('%8.1f %6.1f %s%s'%(s,du,a['Function'],x))
