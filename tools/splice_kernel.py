"""Replace the fifo_kernel template in mcs_kernels.hip with the body in the given file."""
import sys
p = 'multi-cluster-simulator_amd/csrc/mcs_kernels.hip'
s = open(p).read()
i = s.index('template <int NPL, int P>\n__global__ __launch_bounds__(64) void fifo_kernel(FifoArgs a) {')
j = s.index('// ---- variant table')
s = s[:i] + open(sys.argv[1]).read() + s[j:]
open(p, 'w').write(s)
