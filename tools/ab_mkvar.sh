mkvar () 
{ 
    rm -rf /tmp/vv;
    mkdir -p /tmp/vv/a/b /tmp/vv/include;
    cp lsm-kv-storage_amd/csrc/*.h lsm-kv-storage_amd/csrc/sstc_kernels.hip /tmp/vv/a/b/;
    cp include/sstcodec.h /tmp/vv/include/;
    python3 -c "
import sys; p='/tmp/vv/a/b/sstc_kernels.hip'; s=open(p).read(); exec(open('/tmp/edit_$1.py').read()); open(p,'w').write(s)";
    mkdir -p $L/ab/$1;
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -c /tmp/vv/a/b/sstc_kernels.hip -o $L/ab/$1/sstc_kernels.hip.o || return 1;
    objs="";
    for o in $L/obj/*.o;
    do
        b=$(basename $o);
        if [ "$b" = "sstc_kernels.hip.o" ]; then
            objs="$objs $L/ab/$1/sstc_kernels.hip.o";
        else
            objs="$objs $o";
        fi;
    done;
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $L/ab/$1/libsstcodec.so $objs && echo "built $1"
}
