!
! test_shim -- a Fortran host driving the engine through mod_gpu_dyn only (used by
! tests/test_fortran_shim.py).  It runs a script of C-ABI calls that the test writes, the
! calls a RegCM host makes around the dyn step (Main/mod_regcm_interface.F90:150-228:
! the state put, the init bdyval, nsteps x (tend + bdyval) or the physics split of tend,
! bdyin after read_icbc, the 3-hourly sums, restarts), and writes every result it reads back
! to a stream file, so the test can compare it with the Python host running the same script.
!
! Input (stream): int32 size of rcmdyn_config, its memory image, then ops (int32 code + args).
! A code of 24 makes the next op report its return code and message instead of aborting.
!
program test_shim
  use iso_c_binding
  use mod_gpu_dyn
  implicit none
  type(rcmdyn_config), target :: cfg
  type(c_ptr) :: h
  integer(c_int32_t) :: op, dims, fid, j1, j2, i1, i2, k1, k2, n, m, csz
  integer(c_int32_t) :: cpus(2), ext(8), bdy(4)
  integer(c_int) :: ierr
  real(c_double), pointer, contiguous :: a3(:,:,:), a2(:,:)
  real(c_double) :: d3(3), d4(4), ms
  character(len=512) :: fin, fout
  character(kind=c_char) :: info(1024)
  character(kind=c_char), allocatable :: names(:)
  integer(c_int8_t), allocatable :: raw(:)
  integer(c_int64_t) :: lcount, cnt
  integer(c_int64_t), allocatable :: plan(:)
  integer(c_int32_t), allocatable :: launches(:), shares(:)
  real(c_double), allocatable :: avg(:)
  real(c_double) :: dt, xbc
  logical :: soft

  call get_command_argument(1, fin)
  if ( trim(fin) == '--sizeof' ) then
    print '(i0)', c_sizeof(cfg)
    stop
  end if
  call get_command_argument(2, fout)
  open(10, file=trim(fin), access='stream', form='unformatted', status='old')
  open(11, file=trim(fout), access='stream', form='unformatted', status='replace')
  read(10) csz
  if ( csz /= c_sizeof(cfg) ) then
    write(0,*) 'test_shim: rcmdyn_config is ', c_sizeof(cfg), ' bytes here, ', csz, ' in the script'
    error stop 2
  end if
  allocate(raw(csz))
  read(10) raw           ! the C struct's memory image (with its alignment padding)
  cfg = transfer(raw, cfg)
  h = c_null_ptr
  soft = .false.
  do
    read(10) op
    ierr = 0
    select case ( op )
    case ( 0 )
      exit
    case ( 24 )
      soft = .true.
      cycle
    case ( 1 )
      ierr = rcmdyn_create(cfg, h)
    case ( 2 )
      ierr = rcmdyn_destroy(h)
      h = c_null_ptr
    case ( 3, 4 )
      ! put / get of a(j1:j2,i1:i2[,k1:k2]) with the host's own bounds, like getmem*
      read(10) dims, fid, j1, j2, i1, i2, k1, k2
      if ( dims == 2 ) then
        allocate(a2(j1:j2,i1:i2))
        if ( op == 3 ) then
          read(10) a2
          if ( soft ) then
            ierr = rcmdyn_put(h, fid, a2, j1, j2, i1, i2, 1, 1)
          else
            call gpu_put2d(h, fid, a2)
          end if
        else
          a2 = 0.0_c_double
          if ( soft ) then
            ierr = rcmdyn_get(h, fid, a2, j1, j2, i1, i2, 1, 1)
          else
            call gpu_get2d(h, fid, a2)
            write(11) a2
          end if
        end if
        deallocate(a2)
      else
        allocate(a3(j1:j2,i1:i2,k1:k2))
        if ( op == 3 ) then
          read(10) a3
          if ( soft ) then
            ierr = rcmdyn_put(h, fid, a3, j1, j2, i1, i2, k1, k2)
          else
            call gpu_put3d(h, fid, a3)
          end if
        else
          a3 = 0.0_c_double
          if ( soft ) then
            ierr = rcmdyn_get(h, fid, a3, j1, j2, i1, i2, k1, k2)
          else
            call gpu_get3d(h, fid, a3)
            write(11) a3
          end if
        end if
        deallocate(a3)
      end if
    case ( 5 )
      ierr = rcmdyn_tend(h)
    case ( 6 )
      ierr = rcmdyn_bdyval(h)
    case ( 7 )
      read(10) n
      ierr = rcmdyn_step(h, n)
    case ( 8 )
      ierr = rcmdyn_tend_pre_physics(h)
    case ( 9 )
      ierr = rcmdyn_tend_post_physics(h)
    case ( 10 )
      ierr = rcmdyn_bdyin(h)
    case ( 11 )
      ierr = rcmdyn_synchronize(h)
    case ( 12 )
      read(10) lcount, dt, xbc
      ierr = rcmdyn_set_time(h, lcount, dt, xbc)
    case ( 13 )
      ierr = rcmdyn_get_time(h, lcount, dt, xbc)
      if ( ierr == 0 ) write(11) lcount, dt, xbc
    case ( 14 )
      read(10) n
      ierr = rcmdyn_set_diagnostics(h, n)
    case ( 15 )
      ierr = rcmdyn_reductions(h, d3)
      if ( ierr == 0 ) write(11) d3
    case ( 16 )
      ierr = rcmdyn_diagnostics(h, d4)
      if ( ierr == 0 ) write(11) d4
    case ( 17 )
      ierr = rcmdyn_last_step_ms(h, ms)
      if ( ierr == 0 ) write(11) ms
    case ( 18 )
      info = c_null_char
      ierr = rcmdyn_runtime_info(info, 1024)
      if ( ierr == 0 ) write(11) info
    case ( 19 )
      read(10) n, j1, i1
      ierr = rcmdyn_set_nproc(n, j1, i1, cpus)
      if ( ierr == 0 ) write(11) cpus
    case ( 20 )
      read(10) j1, i1, n, m, k1
      ierr = rcmdyn_tile_extent(j1, i1, n, m, k1, ext, bdy)
      if ( ierr == 0 ) write(11) ext, bdy
    case ( 25 )
      ! the extents of tile n of cfg's decomposition, with its periodic directions
      read(10) n
      ierr = rcmdyn_tile_extent_cfg(cfg, n, ext, bdy)
      if ( ierr == 0 ) write(11) ext, bdy
    case ( 21 )
      ! the plan of rank cfg%comm_rank: size it, then fetch it
      read(10) n
      allocate(plan(7))
      ierr = rcmdyn_exchange_plan(cfg, n, plan, 0_c_int64_t, cnt)
      deallocate(plan)
      if ( ierr == 0 ) then
        allocate(plan(7*max(cnt,1_c_int64_t)))
        ierr = rcmdyn_exchange_plan(cfg, n, plan, cnt, cnt)
        if ( ierr == 0 ) write(11) cnt, plan(1:7*cnt)
        deallocate(plan)
      end if
    case ( 22 )
      read(10) n
      allocate(shares(6*n))
      ierr = rcmdyn_overlap_shares(cfg, shares, n)
      if ( ierr == 0 ) write(11) shares
      deallocate(shares)
    case ( 23 )
      read(10) n
      m = 64
      allocate(names(48*m), launches(m), avg(m))
      ierr = rcmdyn_kernel_times(h, n, m, names, launches, avg, k1)
      if ( ierr == 0 ) write(11) k1, launches(1:k1), names(1:48*k1)
      deallocate(names, launches, avg)
    case default
      write(0,*) 'test_shim: unknown op ', op
      error stop 3
    end select
    if ( soft ) then
      ! report instead of aborting: the return code and the engine's message
      info = c_null_char
      if ( ierr /= 0 ) call copy_error(h, info)
      write(11) int(ierr, c_int32_t), info
      soft = .false.
    else
      call gpu_dyn_check(h, ierr, 'op')
    end if
  end do
  close(10)
  close(11)

  contains

  subroutine copy_error(h, buf)
    type(c_ptr), intent(in) :: h
    character(kind=c_char), intent(inout) :: buf(1024)
    character(kind=c_char), pointer :: msg(:)
    integer :: q
    call c_f_pointer(rcmdyn_last_error(h), msg, [1024])
    do q = 1 , 1023
      if ( msg(q) == c_null_char ) exit
      buf(q) = msg(q)
    end do
  end subroutine copy_error

end program test_shim
