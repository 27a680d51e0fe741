// Layout probe for v_mfma_i32_16x16x64_i8 on gfx950: A row = lane&15, B col = lane&15,
// 16 bytes per lane = k 16*(lane>>4)..+15 (any consistent k order), C col = lane&15,
// candidate C rows: 4*(lane>>4)+r  vs  (lane>>4)+4r.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
typedef int v4i __attribute__((ext_vector_type(4)));
__global__ void k(const v4i* a, const v4i* b, v4i* c){
  int l = threadIdx.x; v4i acc = {0,0,0,0};
  acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[l], b[l], acc, 0,0,0);
  c[l] = acc;
}
int main(){
  srand(3);
  int8_t A[16][64], B[64][16]; int C[16][16];
  for(int i=0;i<16;i++) for(int kk=0;kk<64;kk++){ A[i][kk]=rand()%7-3; B[kk][i]=rand()%5-2; }
  for(int i=0;i<16;i++) for(int j=0;j<16;j++){ int s=0; for(int kk=0;kk<64;kk++) s+=A[i][kk]*B[kk][j]; C[i][j]=s; }
  std::vector<int8_t> pa(64*16), pb(64*16);
  for(int l=0;l<64;l++) for(int j=0;j<16;j++){ int kk=16*(l>>4)+j; pa[l*16+j]=A[l&15][kk]; pb[l*16+j]=B[kk][l&15]; }
  v4i *da,*db,*dc; hipMalloc(&da,1024); hipMalloc(&db,1024); hipMalloc(&dc,1024);
  hipMemcpy(da,pa.data(),1024,hipMemcpyHostToDevice); hipMemcpy(db,pb.data(),1024,hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k,dim3(1),dim3(64),0,0,da,db,dc); hipDeviceSynchronize();
  std::vector<int> o(256); hipMemcpy(o.data(),dc,1024,hipMemcpyDeviceToHost);
  for(int cand=0;cand<2;cand++){ int bad=0;
    for(int l=0;l<64;l++) for(int r=0;r<4;r++){ int row = cand==0 ? 4*(l>>4)+r : (l>>4)+4*r; if(o[l*4+r]!=C[row][l&15]) bad++; }
    printf("i8_16x16x64 C cand%d (%s): %s (%d bad)\n",cand,cand==0?"row=4(l>>4)+r":"row=(l>>4)+4r",bad?"FAIL":"PASS",bad); }
  return 0;
}
