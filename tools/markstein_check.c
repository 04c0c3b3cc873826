// Markstein division check (CPU): q = RN(a*y), y = RN(1/b), one and two corrections
// q <- fma(fma(-q, b, a), y, q) against the IEEE quotient a / b, random a, b (sptrsv_grid_kernel).
// gcc -O2 -mfma tools/markstein_check.c -lm -o /tmp/mk && /tmp/mk 200000000
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
static uint64_t s=88172645463325252ull;
static inline uint64_t xr(void){s^=s<<13;s^=s>>7;s^=s<<17;return s;}
static inline double rd(int emin,int erange){uint64_t m=xr()&((1ull<<52)-1);int e=emin+(int)(xr()%erange);uint64_t b=((uint64_t)(e+1023)<<52)|m; if(xr()&1)b|=1ull<<63; double d; memcpy(&d,&b,8); return d;}
int main(int argc,char**argv){long N=atol(argv[1]);long bad1=0,bad2=0;
 for(long i=0;i<N;i++){double a=rd(-30,60),b=rd(-10,20);double q=a/b;double y=1.0/b;
  double q0=a*y;double r0=fma(-q0,b,a);double q1=fma(r0,y,q0);
  if(q1!=q)bad1++;
  double r1=fma(-q1,b,a);double q2=fma(r1,y,q1); if(q2!=q)bad2++;}
 printf("N=%ld one-step mismatches %ld, two-step %ld\n",N,bad1,bad2);}
