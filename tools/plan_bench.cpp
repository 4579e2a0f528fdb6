#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>
#include <algorithm>
#include "ba_plan.h"
using namespace miba;
static double now(){return std::chrono::duration<double,std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();}
int main(int argc,char**argv){
  int nc=atoi(argv[1]), np=atoi(argv[2]), k=atoi(argv[3]);
  std::vector<int> oc, op; std::vector<double> uv, dep;
  std::mt19937 g(1);
  for(int i=0;i<np;++i){int start=(long long)i*(nc-k+1)/np; for(int j=0;j<k;++j){oc.push_back(start+j);op.push_back(i);uv.push_back((float)(g()%640));uv.push_back((float)(g()%480));dep.push_back((float)(1+(g()%1000)/300.0));}}
  int no=oc.size();
  PlanInput in; in.nc=nc; in.np=np; in.no=no; in.fixed_cam=0; in.obs_cam=oc.data(); in.obs_pt=op.data(); in.obs_depth=dep.data(); in.obs_uv=uv.data();
  for(int rep=0;rep<5;++rep){
    Plan pl; double t0=now();
    plan_count(in,pl); double t1=now();
    std::vector<int> seen(nc); for(int i=0;i<nc;++i) seen[i]=pl.cam_cnt[i]>0;
    PlanParams pp; pp.tile_slots=512; pp.subseg = no>=200000?1700:1024;
    plan_order(in,seen,pp,pl); double t2=now();
    plan_envelope(pl); double t3=now();
    printf("threads %d count %.3f order %.3f env %.3f total %.3f ms\n",host_threads(),t1-t0,t2-t1,t3-t2,t3-t0);
  }
}
