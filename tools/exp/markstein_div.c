// Exactness of the division with a shared reciprocal used by the projection (gsm_device.h div_many):
// y = RN(1/b), q = RN(a y), r = fma(-q, b, a), q' = r == 0 ? q : fma(r, y, q) against IEEE a / b, on
// random float pairs (mode 0: any normal numerator, divisor exponents within 2^+-60; mode 1: a in [-b, b]
// with signed zeros; mode 2: fp16-valued numerators; mode 3: arbitrary bit patterns -- zeros, subnormals,
// inf, NaN -- over any positive divisor, with the edges of the fast range).  Pairs outside the fast range
// of div_many (numerators zero or of magnitude in [2^-96, 2^96], divisors in [2^-29, 2^29]) go to the
// division itself and are skipped; every pair inside must match IEEE a / b bit for bit, with nothing
// else skipped (r05: no overflowing or subnormal quotient can reach the fast path).
// usage: gcc -O2 -ffp-contract=off markstein_div.c -lm && ./a.out N MODE
// (prints "bad 0" when every quotient matched; tests/test_markstein_div.py runs it on the CPU).
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static inline float bf(uint32_t u){float f; memcpy(&f,&u,4); return f;}
static uint64_t s=88172645463325252ull;
static inline uint64_t rnd(){ s^=s<<13; s^=s>>7; s^=s<<17; return s; }
static inline float dv(float a, float y, float b){ float q=a*y; float r=fmaf(-q,b,a); return r==0.0f? q : fmaf(r,y,q); }
static inline int slow(float a){ uint32_t x; memcpy(&x,&a,4); x&=0x7FFFFFFFu; return x!=0u && x-(31u<<23) > (192u<<23); }
int main(int argc,char**argv){
  long N=atol(argv[1]); int mode=atoi(argv[2]); s+=mode*7919;
  long bad=0, tested=0;
  for(long i=0;i<N;i++){
    uint64_t r=rnd();
    float a,b;
    if(mode==0){ uint32_t ea=(uint32_t)(1+(r%253)), eb=(uint32_t)(127-60+((r>>8)%121));
      a=bf((ea<<23)|((uint32_t)(r>>16)&0x7FFFFF)|(((r>>40)&1)<<31));
      b=bf((eb<<23)|((uint32_t)(r>>20)&0x7FFFFF)); }
    else if(mode==1){ b=bf(((uint32_t)(127-27+(r%40))<<23)|((uint32_t)(r>>16)&0x7FFFFF));
      float t=(float)((r>>40)&0xFFFFFF)/16777216.0f*2.0f-1.0f; a=t*b; if(((r>>60)&7)==0) a=((r>>59)&1)? -0.0f: 0.0f; }
    else if(mode==3){ // any bit pattern over any positive divisor; a quarter of each at the range edges
      uint32_t ua=(uint32_t)(r>>32), ub=(uint32_t)r & 0x7FFFFFFFu;
      if(((r>>20)&3)==0){ static const uint32_t ea[]={0u,(31u<<23),(31u<<23)-1u,(223u<<23),(223u<<23)+1u,0x7F800000u,0x7FC00000u,1u};
        ua=(ua&0x80000000u)|(ea[(r>>22)&7]+(uint32_t)((r>>25)&3)); }
      if(((r>>28)&3)==0){ static const uint32_t eb[]={(98u<<23),(156u<<23),(98u<<23)-1u,(156u<<23)+1u};
        ub=eb[(r>>30)&3]+(uint32_t)((r>>33)&7); }
      a=bf(ua); b=bf(ub); if(!(b>0.0f)) continue; }
    else { // fp16-valued numerators (quaternion / direction components) over a norm
      uint32_t h=(uint32_t)(r>>16)&0xFFFF; uint32_t e=(h>>10)&31, m=h&1023, sg=(h>>15)&1; if(e==31) continue;
      a = (e==0? ldexpf((float)m, -24) : ldexpf((float)(m|1024), (int)e-25)); if(sg) a=-a;
      b=bf(((uint32_t)(127-27+(r%60))<<23)|((uint32_t)(r>>32)&0x7FFFFF)); }
    if(slow(a) || !(b>=0x1p-29f && b<=0x1p29f)) continue;  // (div_many divides these)
    float y=1.0f/b;
    float q2=dv(a,y,b), ref=a/b;
    tested++;
    if(memcmp(&q2,&ref,4)!=0){ if(bad<5) printf("a=%a b=%a q2=%a ref=%a\n",a,b,q2,ref); bad++; }
  }
  printf("mode %d N %ld tested %ld bad %ld\n",mode,N,tested,bad);
  return 0;
}
