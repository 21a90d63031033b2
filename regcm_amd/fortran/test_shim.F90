!
! test_shim -- Fortran host driver exercising mod_gpu_dyn end to end (used by
! tests/test_fortran_shim_gpu.py).  Mirrors the RCM_run loop (Main/mod_regcm_interface.F90:
! 172-228) with physics stubbed: bdyval once at init, then nsteps x (tend + bdyval).
! Input/output are raw stream files written/read by the test.
!
program test_shim
  use iso_c_binding
  use mod_gpu_dyn
  implicit none
  type(rcmdyn_config), target :: cfg
  type(c_ptr) :: h
  integer(c_int32_t) :: jx, iy, kz, nsplit, nsteps, nf, fid, nk, n, s
  real(c_double), pointer, contiguous :: a3(:,:,:), a2(:,:)
  real(c_double), pointer, contiguous :: t(:,:,:), u(:,:,:), ps(:,:)
  character(len=512) :: fin, fout
  integer(c_int8_t), allocatable :: raw(:)
  integer(c_int64_t) :: lcount
  real(c_double) :: dt, xbc
  call get_command_argument(1, fin)
  if ( trim(fin) == '--sizeof' ) then
    print '(i0)', c_sizeof(cfg)
    stop
  end if
  call get_command_argument(2, fout)
  if ( trim(fin) == '--dump' ) then
    open(10, file=trim(fout), access='stream', form='unformatted', status='old')
    read(10) jx, iy, kz, nsplit, nsteps
    allocate(raw(c_sizeof(cfg)))
    read(10) raw         ! the C struct's memory image (with its alignment padding)
    cfg = transfer(raw, cfg)
    close(10)
    print *, cfg%jx, cfg%kz, cfg%dtsec, cfg%pd, cfg%device, cfg%comm_size, cfg%nsplit
    stop
  end if
  open(10, file=trim(fin), access='stream', form='unformatted', status='old')
  read(10) jx, iy, kz, nsplit, nsteps
  allocate(raw(c_sizeof(cfg)))
  read(10) raw           ! the C struct's memory image (with its alignment padding)
  cfg = transfer(raw, cfg)
  call gpu_dyn_check(c_null_ptr, rcmdyn_create(cfg, h), 'create')
  read(10) nf
  do n = 1 , nf
    read(10) fid, nk
    if ( nk == 1 ) then
      ! p* style 2-D array with a one-point ghost ring, like getmem2d(jce1ga:jce2ga,...)
      allocate(a2(0:jx+1,0:iy+1))
      a2 = 0.0_c_double
      read(10) a2(1:jx,1:iy)
      call gpu_put2d(h, fid, a2)
      deallocate(a2)
    else
      allocate(a3(1:jx,1:iy,1:nk))
      read(10) a3
      call gpu_put3d(h, fid, a3)
      deallocate(a3)
    end if
  end do
  close(10)
  call gpu_dyn_check(h, rcmdyn_bdyval(h), 'bdyval')
  do s = 1 , nsteps
    call gpu_dyn_check(h, rcmdyn_tend(h), 'tend')
    call gpu_dyn_check(h, rcmdyn_bdyval(h), 'bdyval')
  end do
  allocate(t(1:jx,1:iy,1:kz), u(1:jx,1:iy,1:kz), ps(1:jx,1:iy))
  t = 0.0_c_double ; u = 0.0_c_double ; ps = 0.0_c_double
  call gpu_get3d(h, f_atm1_t, t)
  call gpu_get3d(h, f_atm1_u, u)
  call gpu_get2d(h, f_psa, ps)
  call gpu_dyn_check(h, rcmdyn_get_time(h, lcount, dt, xbc), 'get_time')
  open(11, file=trim(fout), access='stream', form='unformatted', status='replace')
  write(11) lcount, dt, xbc
  write(11) t, u, ps
  close(11)
  call gpu_dyn_check(h, rcmdyn_destroy(h), 'destroy')
end program test_shim
