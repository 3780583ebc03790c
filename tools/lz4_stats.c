/* lz4_stats.c — how often the greedy LZ4 parse (lz4 r123 LZ4_compress, byU32, the loop of
 * oracle/hdrf_oracle.c hdrf_oracle_lz4_compress with counters added) loads a candidate whose 4 bytes
 * differ from the bytes being matched, and how many of those a k-bit tag from the hash product would
 * reject.  CPU measurement tool, not part of the product or the oracle.
 *   gcc -O2 tools/lz4_stats.c -o /tmp/lz4_stats && /tmp/lz4_stats segments.bin
 * segments.bin: raw bytes cut into 261,100-B segments (e.g. config-4 corpus segments of one kind). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static uint32_t rd(const uint8_t *p){uint32_t v;memcpy(&v,p,4);return v;}
typedef struct { long seq, att, att_in, att_match, att_tagpass[5], chain, chain_in, chain_match, chain_tagpass[5], mlen, lits; long dist_hist[8]; } st;
static int tagpass(uint32_t a, uint32_t b, int k){ uint32_t ha=(a*2654435761u)>>(20-k), hb=(b*2654435761u)>>(20-k); return ((ha^hb)&((1u<<k)-1))==0; }
static void dist(st*s,long d){int b=0; while(d>=256 && b<7){d>>=2;b++;} s->dist_hist[b]++;}
void run(const uint8_t *src, long n, st *s){
  const int hlog=12; uint32_t *table=calloc(1<<hlog,4);
  const uint8_t *ip=src,*anchor=src,*iend=src+n,*mflimit=iend-12,*matchlimit=iend-5;
#define H(p) ((rd(p)*2654435761u)>>(32-hlog))
  table[H(ip)]=0; ip++; uint32_t fh=H(ip);
  for(;;){ int attempts=67; const uint8_t *fip=ip,*ref;
    for(;;){ uint32_t h=fh; int step=attempts++>>6; ip=fip; fip=ip+step; if(fip>mflimit) goto done; fh=H(fip); ref=src+table[h]; table[h]=ip-src;
      s->att++; int in = !(ref+65535<ip); if(in){ s->att_in++; dist(s, ip-ref); int m=rd(ref)==rd(ip); s->att_match+=m; for(int k=1;k<=4;k++) s->att_tagpass[k]+= (!m && tagpass(rd(ref),rd(ip),k)); if(m) break; } }
    while(ip>anchor && ref>src && ip[-1]==ref[-1]){ip--;ref--;}
    s->lits += ip-anchor;
  next:
    s->seq++;
    ip+=4; ref+=4; anchor=ip; while(ip<matchlimit && *ip==*ref){ip++;ref++;}
    s->mlen += ip-anchor+4;
    if(ip>mflimit){anchor=ip;break;}
    table[H(ip-2)]=ip-2-src; ref=src+table[H(ip)]; table[H(ip)]=ip-src;
    s->chain++; if(ref+65535>=ip){ s->chain_in++; dist(s, ip-ref); int m=rd(ref)==rd(ip); s->chain_match+=m; for(int k=1;k<=4;k++) s->chain_tagpass[k]+=(!m && tagpass(rd(ref),rd(ip),k)); if(m) goto next; }
    anchor=ip++; fh=H(ip);
  }
done: free(table);
}
int main(int argc,char**argv){
  FILE*f=fopen(argv[1],"rb"); fseek(f,0,2); long n=ftell(f); fseek(f,0,0); uint8_t*b=malloc(n); if(fread(b,1,n,f)!=(size_t)n) return 1;
  st s; memset(&s,0,sizeof s); long seg=261100; for(long o=0;o+seg<=n;o+=seg) run(b+o,seg,&s);
  printf("segs %ld seq %ld avg_mlen %.1f lits/seq %.1f\n", n/seg, s.seq, (double)s.mlen/s.seq, (double)s.lits/s.seq);
  printf("search: att %ld (%.1f/seq) in-dist %ld match %ld  false-in-dist %ld tagpass k1..4: %ld %ld %ld %ld\n", s.att,(double)s.att/s.seq,s.att_in,s.att_match,s.att_in-s.att_match,s.att_tagpass[1],s.att_tagpass[2],s.att_tagpass[3],s.att_tagpass[4]);
  printf("chain: %ld in-dist %ld match %ld false %ld tagpass k1..4: %ld %ld %ld %ld\n", s.chain,s.chain_in,s.chain_match,s.chain_in-s.chain_match,s.chain_tagpass[1],s.chain_tagpass[2],s.chain_tagpass[3],s.chain_tagpass[4]);
  printf("dist hist (<256,<1K,<4K,<16K,<64K..):"); for(int i=0;i<8;i++) printf(" %ld",s.dist_hist[i]); printf("\n");
}
