// Website shell: top navigation, identity menu and the client router (the reference's Website/Website/client:
// package.loader.js resolves web.composition.json pages to package components; topNav*.jsx from datax-common).
// A page is {routePath, packageName, componentName, componentProps}; its component is
// `export function <componentName>(props, ctx)` of /dist/<packageName>/index.js, returning an element.
import { h, mount } from './common/dom.js';
import { nodeGet, getToken, setToken } from './common/api.js';
import { userContext, MessageBar } from './common/components.js';

let composition = null;
let current = null; // {page, dispose}

export function matchRoute(pattern, path) {
    const ps = pattern.split('/').filter(Boolean);
    const xs = path.split('/').filter(Boolean);
    if (ps.length !== xs.length) return null;
    const params = {};
    for (let i = 0; i < ps.length; i++) {
        if (ps[i].startsWith(':')) params[ps[i].slice(1)] = decodeURIComponent(xs[i]);
        else if (ps[i] !== xs[i]) return null;
    }
    return params;
}

export function resolvePage(pages, path) {
    // exact patterns win over parameterised ones ('/config/new' before '/config/edit/:id')
    const enabled = pages.filter(p => p.enable && !p.externalUrl);
    const ordered = enabled.filter(p => !p.routePath.includes(':')).concat(enabled.filter(p => p.routePath.includes(':')));
    for (const p of ordered) {
        const params = matchRoute(p.routePath, path);
        if (params) return { page: p, params };
    }
    return null;
}

export function navigate(path, replace) {
    if (replace) history.replaceState({}, '', path);
    else history.pushState({}, '', path);
    route();
}

async function route() {
    const path = location.pathname === '/' ? '/home' : location.pathname;
    const m = resolvePage(composition.pages, path);
    const host = document.getElementById('page');
    if (current && current.dispose) current.dispose();
    current = null;
    renderNav(m ? m.page : null);
    if (!m) {
        mount(host, MessageBar('error', `No page at ${path}`));
        return;
    }
    try {
        const mod = await import(`./${m.page.packageName}/index.js`);
        const comp = mod[m.page.componentName];
        if (!comp) throw new Error(`package ${m.page.packageName} has no component ${m.page.componentName}`);
        const ctx = { navigate, params: m.params, page: m.page, onDispose: fn => (current.dispose = fn) };
        current = { page: m.page, dispose: null };
        const el = comp(Object.assign({}, m.page.componentProps || {}, m.params), ctx);
        mount(host, el);
    } catch (e) {
        mount(host, MessageBar('error', `Failed to load ${m.page.packageName}: ${e.message}`));
    }
}

function renderNav(active) {
    const nav = document.getElementById('topnav');
    const byKey = {};
    for (const p of composition.pages) byKey[p.key] = p;
    const links = (composition.nav || []).map(k => byKey[k]).filter(p => p && p.enable);
    let menuOpen = false;
    const menu = h('div', { class: 'menu', hidden: true });
    const identity = h(
        'div',
        {
            class: 'identity',
            onclick: e => {
                if (e.target.closest('.menu')) return;
                menuOpen = !menuOpen;
                menu.hidden = !menuOpen;
            }
        },
        (userContext.user.name || 'anonymous') + (userContext.user.isWriter ? ' (writer)' : ' (reader)'),
        menu
    );
    const tokenBox = h('textarea', { class: 'mono', placeholder: 'Azure AD / JWT bearer token', value: getToken() });
    mount(
        menu,
        h('div', null, h('b', null, userContext.user.name || 'anonymous')),
        h('div', { class: 'muted' }, 'roles: ' + ((userContext.user.roles || []).join(', ') || 'none')),
        h('div', { class: 'muted' }, 'auth mode: ' + (userContext.user.authMode || 'unknown')),
        h('p', null, 'Bearer token (sent with every API call):'),
        tokenBox,
        h(
            'div',
            { class: 'row' },
            h('button', { class: 'primary', onclick: () => { setToken(tokenBox.value.trim()); location.reload(); } }, 'Sign in'),
            h('button', { onclick: () => { setToken(''); location.reload(); } }, 'Sign out')
        )
    );
    mount(
        nav,
        h('span', { class: 'brand' }, composition.displayName || 'Data Accelerator'),
        links.map(p =>
            h(
                'a',
                {
                    href: p.routePath,
                    class: active && active.title === p.title ? 'on' : '',
                    onclick: e => {
                        e.preventDefault();
                        navigate(p.routePath);
                    }
                },
                p.title
            )
        ),
        identity
    );
}

async function boot() {
    composition = await nodeGet('web-composition');
    try {
        userContext.user = await nodeGet('user');
        userContext.functions = await nodeGet('functionenabled');
    } catch (e) {
        userContext.user = { name: 'not signed in', roles: [], isWriter: false, error: e.message };
        userContext.functions = {};
    }
    try {
        userContext.enableLocalOneBox = (await nodeGet('enableLocalOneBox')).enableLocalOneBox;
    } catch (e) {
        userContext.enableLocalOneBox = false;
    }
    window.addEventListener('popstate', route);
    // in-page links: <a data-nav href="/x">
    document.addEventListener('click', e => {
        const a = e.target.closest && e.target.closest('a[data-nav]');
        if (a) {
            e.preventDefault();
            navigate(a.getAttribute('href'));
        }
    });
    await route();
}

if (typeof window !== 'undefined' && typeof document !== 'undefined' && document.getElementById('page')) {
    boot().catch(e => mount(document.getElementById('page'), MessageBar('error', 'Website failed to start: ' + e.message)));
}
