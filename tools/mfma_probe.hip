// MFMA operand/result layout probe for gfx950 (i8 32x32x32, f64 16x16x4).
// Packs A/B per candidate lane map on the host, runs one MFMA, checks the
// result against a CPU product under the candidate C/D map. Prints PASS/FAIL.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef double v4d __attribute__((ext_vector_type(4)));
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP err %s line %d\n",hipGetErrorString(e),__LINE__); exit(1);}}while(0)

__global__ void k_i8(const v4i* a, const v4i* b, v16i* c){
  int l = threadIdx.x; v16i acc = {};
  acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[l], b[l], acc, 0,0,0);
  c[l] = acc;
}
__global__ void k_f64(const double* a, const double* b, v4d* y){
  int l = threadIdx.x; v4d d = {};
  d = __builtin_amdgcn_mfma_f64_16x16x4f64(a[l], b[l], d, 0,0,0);
  y[l] = d;
}

int main(){
  srand(7);
  // ---- i8 32x32x32 ----
  int8_t A[32][32], B[32][32]; int C[32][32];
  for(int i=0;i<32;i++) for(int k=0;k<32;k++){ A[i][k]=rand()%7-3; B[k][i]=rand()%5-2; }
  for(int i=0;i<32;i++) for(int j=0;j<32;j++){ int s=0; for(int k=0;k<32;k++) s+=A[i][k]*B[k][j]; C[i][j]=s; }
  v4i *da,*db; v16i* dc; CK(hipMalloc(&da,64*16)); CK(hipMalloc(&db,64*16)); CK(hipMalloc(&dc,64*64));
  for(int cand=0;cand<2;cand++){
    std::vector<int8_t> pa(64*16), pb(64*16);
    for(int l=0;l<64;l++) for(int j=0;j<16;j++){
      int k = cand==0 ? 16*(l>>5)+j : (j<8 ? 8*(l>>5)+j : 16+8*(l>>5)+(j-8));
      pa[l*16+j]=A[l&31][k]; pb[l*16+j]=B[k][l&31];
    }
    CK(hipMemcpy(da,pa.data(),1024,hipMemcpyHostToDevice)); CK(hipMemcpy(db,pb.data(),1024,hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_i8,dim3(1),dim3(64),0,0,da,db,dc); CK(hipDeviceSynchronize());
    std::vector<int> out(64*16); CK(hipMemcpy(out.data(),dc,64*64,hipMemcpyDeviceToHost));
    int bad=0;
    for(int l=0;l<64;l++) for(int r=0;r<16;r++){ int row=(r&3)+8*(r>>2)+4*(l>>5), col=l&31; if(out[l*16+r]!=C[row][col]) bad++; }
    printf("i8_32x32x32 cand%d (%s): %s (%d bad)\n",cand,cand==0?"k=16h+j":"k=8h+j|16+8h+j",bad?"FAIL":"PASS",bad);
  }
  // ---- f64 16x16x4 ----
  double Af[16][4], Bf[4][16], Cf[16][16];
  for(int i=0;i<16;i++) for(int k=0;k<4;k++){ Af[i][k]=rand()%9-4; Bf[k][i]=rand()%11-5; }
  for(int i=0;i<16;i++) for(int j=0;j<16;j++){ double s=0; for(int k=0;k<4;k++) s+=Af[i][k]*Bf[k][j]; Cf[i][j]=s; }
  double *fa,*fb; v4d* fy; CK(hipMalloc(&fa,512)); CK(hipMalloc(&fb,512)); CK(hipMalloc(&fy,64*32));
  std::vector<double> qa(64), qb(64);
  for(int l=0;l<64;l++){ qa[l]=Af[l&15][l>>4]; qb[l]=Bf[l>>4][l&15]; }
  CK(hipMemcpy(fa,qa.data(),512,hipMemcpyHostToDevice)); CK(hipMemcpy(fb,qb.data(),512,hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_f64,dim3(1),dim3(64),0,0,fa,fb,fy); CK(hipDeviceSynchronize());
  std::vector<double> o(64*4); CK(hipMemcpy(o.data(),fy,64*32,hipMemcpyDeviceToHost));
  for(int cand=0;cand<2;cand++){
    int bad=0;
    for(int l=0;l<64;l++) for(int r=0;r<4;r++){
      int row = cand==0 ? (l>>4)+4*r : 4*(l>>4)+r; int col=l&15;
      if(o[l*4+r]!=Cf[row][col]) bad++;
    }
    printf("f64_16x16x4 C cand%d (%s): %s (%d bad)\n",cand,cand==0?"row=(l>>4)+4r":"row=4(l>>4)+r",bad?"FAIL":"PASS",bad);
  }
  return 0;
}
