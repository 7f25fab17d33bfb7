// Probe (round 6): config 1's per-file gather pattern (cas.rs:23-62 offsets: header + sample 0
// as one read, samples 1-3, fstat, footer) read with pread, as host_paths.cpp does, vs the same
// reads batched through io_uring (raw syscalls, no liburing in the image), on page-cached
// tmpfs files.  Build: gcc -O2 tools/probe_uring.c -o tools/probe_uring; run:
// tools/probe_uring <files> <batch> [dir].  Prints microseconds per file for both forms.
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <fcntl.h>
#include <unistd.h>
#include <sys/stat.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <linux/io_uring.h>
#include <time.h>
#include <string.h>
#include <stdatomic.h>
static double now(){struct timespec t;clock_gettime(CLOCK_MONOTONIC,&t);return t.tv_sec+t.tv_nsec*1e-9;}
struct ring{int fd; unsigned *sq_head,*sq_tail,*sq_mask,*sq_array,*cq_head,*cq_tail,*cq_mask; struct io_uring_sqe*sqes; struct io_uring_cqe*cqes;};
static int ring_init(struct ring*r,unsigned ent){struct io_uring_params p;memset(&p,0,sizeof p);r->fd=syscall(__NR_io_uring_setup,ent,&p);if(r->fd<0)return -1;
 size_t sl=p.sq_off.array+p.sq_entries*4, cl=p.cq_off.cqes+p.cq_entries*sizeof(struct io_uring_cqe);
 char*sq=mmap(0,sl,PROT_READ|PROT_WRITE,MAP_SHARED|MAP_POPULATE,r->fd,IORING_OFF_SQ_RING);
 char*cq=(p.features&IORING_FEAT_SINGLE_MMAP)?sq:mmap(0,cl,PROT_READ|PROT_WRITE,MAP_SHARED|MAP_POPULATE,r->fd,IORING_OFF_CQ_RING);
 if(p.features&IORING_FEAT_SINGLE_MMAP && cl>sl){munmap(sq,sl);sq=cq=mmap(0,cl,PROT_READ|PROT_WRITE,MAP_SHARED|MAP_POPULATE,r->fd,IORING_OFF_SQ_RING);}
 r->sqes=mmap(0,p.sq_entries*sizeof(struct io_uring_sqe),PROT_READ|PROT_WRITE,MAP_SHARED|MAP_POPULATE,r->fd,IORING_OFF_SQES);
 r->sq_head=(unsigned*)(sq+p.sq_off.head);r->sq_tail=(unsigned*)(sq+p.sq_off.tail);r->sq_mask=(unsigned*)(sq+p.sq_off.ring_mask);r->sq_array=(unsigned*)(sq+p.sq_off.array);
 r->cq_head=(unsigned*)(cq+p.cq_off.head);r->cq_tail=(unsigned*)(cq+p.cq_off.tail);r->cq_mask=(unsigned*)(cq+p.cq_off.ring_mask);r->cqes=(struct io_uring_cqe*)(cq+p.cq_off.cqes);return 0;}
static unsigned tail_local;
static void prep(struct ring*r,int op,int fd,void*buf,unsigned len,long off,unsigned long ud){unsigned t=tail_local++;unsigned i=t&*r->sq_mask;struct io_uring_sqe*s=&r->sqes[i];memset(s,0,sizeof*s);s->opcode=op;s->fd=fd;s->addr=(unsigned long)buf;s->len=len;s->off=off;s->user_data=ud;r->sq_array[i]=i;}
static int submit_wait(struct ring*r,unsigned n){atomic_store_explicit((_Atomic unsigned*)r->sq_tail,tail_local,memory_order_release);int ret=syscall(__NR_io_uring_enter,r->fd,n,n,IORING_ENTER_GETEVENTS,0,0);
 unsigned h=*r->cq_head,t=atomic_load_explicit((_Atomic unsigned*)r->cq_tail,memory_order_acquire);int bad=0;while(h!=t){if(r->cqes[h&*r->cq_mask].res<0)bad++;h++;}atomic_store_explicit((_Atomic unsigned*)r->cq_head,h,memory_order_release);return ret<0?ret:bad;}
int main(int argc,char**argv){
  int n=atoi(argv[1]),B=atoi(argv[2]); const char*dir=argc>3?argv[3]:"/dev/shm/sd_probe_uring"; char p[256]; char*buf=malloc((size_t)B*57344);
  char *blk=malloc(1<<20); for(int i=0;i<(1<<20);i++) blk[i]=rand();
  for(int i=0;i<n;i++){sprintf(p,"%s/f%d",dir,i); int fd=open(p,O_CREAT|O_WRONLY|O_TRUNC,0644); if(write(fd,blk,300000+(i*7919)%700000)<0)return 1; close(fd);}
  struct ring r; if(ring_init(&r,8*B)){perror("setup");return 1;}
  int *fds=malloc(n*sizeof(int)); long *sz=malloc(n*sizeof(long));
  for(int rep=0;rep<3;rep++){
  for(int i=0;i<n;i++){sprintf(p,"%s/f%d",dir,i); fds[i]=open(p,O_RDONLY|O_CLOEXEC); struct stat st; fstat(fds[i],&st); sz[i]=st.st_size;}
  double t0=now(); volatile long s=0;
  for(int i=0;i<n;i++){ char*b=buf+(size_t)(i%B)*57344; long j=(sz[i]-16384)/4; s+=pread(fds[i],b,18432,0); for(int k=1;k<4;k++) s+=pread(fds[i],b+8192+k*10240,10240,8192+k*j); struct stat st; fstat(fds[i],&st); s+=pread(fds[i],b+49152,8192,st.st_size-8192);}
  double t1=now(); int bad=0;
  for(int i0=0;i0<n;i0+=B){int m=(n-i0<B)?n-i0:B; for(int q=0;q<m;q++){int i=i0+q;char*b=buf+(size_t)q*57344; long j=(sz[i]-16384)/4; prep(&r,IORING_OP_READ,fds[i],b,18432,0,i); for(int k=1;k<4;k++) prep(&r,IORING_OP_READ,fds[i],b+8192+k*10240,10240,8192+k*j,i); prep(&r,IORING_OP_READ,fds[i],b+49152,8192,sz[i]-8192,i);} int x=submit_wait(&r,5*m); if(x) bad+=x;}
  double t2=now();
  for(int i=0;i<n;i++) close(fds[i]);
  printf("per file us: pread path %.2f  io_uring B=%d %.2f  bad=%d\n",(t1-t0)/n*1e6,B,(t2-t1)/n*1e6,bad);}
  return 0;}
