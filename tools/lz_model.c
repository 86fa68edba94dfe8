// Size model of the device writer's LZ77 parse (measurement tool, not product
// code): per 4 KiB segment, a hash table refreshed once per chunk of CH
// positions (stale within a chunk, as the 256-thread rounds of k_lz_parse),
// DEPTH candidates per bucket, greedy or one-step lazy parse, window W bytes;
// the size is estimated with per-1-MiB-block Huffman codes plus extra bits.
//   gcc -O2 -o lz_model tools/lz_model.c && ./lz_model TEXT CH HBITS LAZY W [DEPTH]
// TEXT: e.g. tools/lz_sample_text.py's output (config-2-like normalised rows).
// GPU-style parse model: per segment, table refreshed per chunk of CH positions (stale within a chunk),
// match finding for all positions in parallel, then greedy (optionally lazy-1) walk.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
static const int lbase[29]={3,4,5,6,7,8,9,10,11,13,15,17,19,23,27,31,35,43,51,59,67,83,99,115,131,163,195,227,258};
static const int lext[29]={0,0,0,0,0,0,0,0,1,1,1,1,2,2,2,2,3,3,3,3,4,4,4,4,5,5,5,5,0};
static const int dbase[30]={1,2,3,4,5,7,9,13,17,25,33,49,65,97,129,193,257,385,513,769,1025,1537,2049,3073,4097,6145,8193,12289,16385,24577};
static const int dext[30]={0,0,0,0,1,1,2,2,3,3,4,4,5,5,6,6,7,7,8,8,9,9,10,10,11,11,12,12,13,13};
static int lsym(int l){int i=28;while(lbase[i]>l)i--;return i;}
static int dsym(int d){int i=29;while(dbase[i]>d)i--;return i;}
static double huff_bits(const long *h, int n){
  long w[600]; int par[600]; int cnt=0; int idx[300];
  for(int i=0;i<n;i++){ if(h[i]){idx[i]=cnt; w[cnt]=h[i]; par[cnt]=-1; cnt++;} else idx[i]=-1; }
  if(cnt<=1){ long t=0; for(int i=0;i<n;i++) t+=h[i]; return t; }
  int alive[600]; int na=cnt; for(int i=0;i<cnt;i++) alive[i]=1; int tot=cnt;
  while(na>1){ int a=-1,b=-1; for(int i=0;i<tot;i++) if(alive[i]){ if(a<0||w[i]<w[a]){b=a;a=i;} else if(b<0||w[i]<w[b]) b=i; }
    alive[a]=alive[b]=0; w[tot]=w[a]+w[b]; par[tot]=-1; alive[tot]=1; par[a]=par[b]=tot; tot++; na--; }
  double bits=0; for(int i=0;i<n;i++) if(idx[i]>=0){ int d=0,k=idx[i]; while(par[k]>=0){k=par[k];d++;} bits+=(double)h[i]*d; }
  return bits;
}
int main(int argc,char**argv){
  FILE*f=fopen(argv[1],"rb"); fseek(f,0,2); long n=ftell(f); fseek(f,0,0); unsigned char*t=malloc(n+16); if(fread(t,1,n,f)!=n) return 1; memset(t+n,0,16);
  int CH=atoi(argv[2]); int hbits=atoi(argv[3]); int lazy=atoi(argv[4]); long W=atol(argv[5]); int SEG=4096; int MINM=4;
  int depth = argc>6?atoi(argv[6]):1;
  int hs=1<<hbits; long *tab=malloc(sizeof(long)*hs*depth); int *ml=malloc(4*SEG), *md=malloc(4*SEG);
  long blk=1<<20; double total=0; long lh[286],dh[30]; double extra;
  for(long b0=0;b0<n;b0+=blk){
    long b1=b0+blk<n?b0+blk:n; memset(lh,0,sizeof lh); memset(dh,0,sizeof dh); extra=0;
    for(long s0=b0;s0<b1;s0+=SEG){
      long s1=s0+SEG<b1?s0+SEG:b1; long ws=s0-W>b0?s0-W:b0;
      for(long i=0;i<hs*depth;i++) tab[i]=-1;
      #define H(p) ((((uint32_t)t[p]|(uint32_t)t[p+1]<<8|(uint32_t)t[p+2]<<16|(uint32_t)t[p+3]<<24)*2654435761u)>>(32-hbits))
      for(long c0=ws;c0<s1;c0+=CH){
        long c1=c0+CH<s1?c0+CH:s1;
        for(long p=c0;p<c1;p++) if(p>=s0){ long bl=0,bd=0; if(p+MINM<=s1){ long*e=tab+H(p)*depth; for(int q=0;q<depth;q++){ long c=e[q]; if(c<0) continue; long l=0; long lim=s1-p<258?s1-p:258; while(l<lim && t[c+l]==t[p+l]) l++; if(l>bl){bl=l;bd=p-c;} } }
          ml[p-s0]=bl>=MINM?bl:0; md[p-s0]=bd; }
        for(long p=c0;p<c1;p++) if(p+4<=b1){ long*e=tab+H(p)*depth; for(int q=depth-1;q>0;q--) e[q]=e[q-1]; e[0]=p; }
      }
      long p=s0;
      while(p<s1){ int i=p-s0; int l=ml[i];
        if(l && lazy && i+1<s1-s0 && ml[i+1]>l) l=0;
        if(l){ lh[257+lsym(l)]++; extra+=lext[lsym(l)]; dh[dsym(md[i])]++; extra+=dext[dsym(md[i])]; p+=l; }
        else { lh[t[p]]++; p++; } }
    }
    lh[256]++; total+=huff_bits(lh,286)+huff_bits(dh,30)+extra+600;
  }
  printf("CH %d hbits %d lazy %d W %ld depth %d: ratio %.4f\n",CH,hbits,lazy,W,depth,total/8/n);
}
