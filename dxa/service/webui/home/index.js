// Home page (datax-home: homePage.jsx, welcomeCard, section/card/wideCard, footerItem; composition.js lists the
// getting-started steps). Cards link to the other packages; the live summary reads flows, jobs and the built-in
// event-rate metric of every flow.
import { h, mount, formatters } from '../common/dom.js';
import { flowApi, jobApi, getMetricsData } from '../common/api.js';
import { userContext, MessageBar } from '../common/components.js';

const STEPS = [
    ['Create a flow', 'Pick an input (Event Hub, IoT Hub, Kafka, Blob or the local generator), infer the schema from ' +
        'live samples and write SQL over DataXProcessedInput.', '/config/new'],
    ['Test it live', 'LiveQuery runs the SQL against sampled events on the GPU while you edit, in the Query tab.', '/config'],
    ['Add rules and outputs', 'Tag and alert rules are built from conditions; outputs go to Blob, Event Hub, Cosmos DB, ' +
        'SQL Server or local files.', '/config'],
    ['Deploy', 'Deploy generates the job config and starts one process per GPU over RCCL; jobs are managed on the Jobs page.', '/jobs'],
    ['Watch it', 'The metrics dashboard charts events/s, latency and your own metric outputs per flow.', '/dashboard']
];

function Card(title, text, href, linkText) {
    return h(
        'div',
        { class: 'card' },
        h('h3', null, title),
        h('p', { class: 'muted' }, text),
        href ? h('a', { href, 'data-nav': true }, linkText || 'Open') : null
    );
}

export function HomePage(props, ctx) {
    const summary = h('div', { class: 'panel' }, h('div', { class: 'muted' }, 'Loading summary...'));
    const root = h(
        'div',
        null,
        h(
            'div',
            { class: 'welcome' },
            h('h2', { style: { margin: '0 0 6px', fontWeight: 500 } }, 'Welcome to Data Accelerator'),
            h('div', null, 'Streaming SQL pipelines on AMD Instinct MI355X GPUs: JSON parsing, SQL, windows, joins and ' +
                'outputs run as HIP kernels; ranks scale over RCCL.'),
            h('div', { style: { marginTop: '8px' } }, 'Signed in as ', h('b', null, userContext.user.name || 'anonymous'),
                userContext.enableLocalOneBox ? ' — local one-box mode' : '')
        ),
        h('div', { class: 'panel-header' }, 'Get started'),
        h('div', { class: 'cards' }, STEPS.map((s, i) => Card(`${i + 1}. ${s[0]}`, s[1], s[2]))),
        h('div', { class: 'panel-header', style: { marginTop: '16px' } }, 'At a glance'),
        summary
    );
    loadSummary(summary);
    return root;
}

async function loadSummary(el) {
    try {
        const [flows, jobs] = await Promise.all([flowApi.getAllMin(), jobApi.getAll()]);
        const running = (jobs || []).filter(j => (j.state || '').toLowerCase() === 'running');
        const now = Date.now();
        const rates = await Promise.all(
            (flows || []).map(async f => {
                const pts = await getMetricsData(`DATAX-${f.name}:Input_DataXProcessedInput_Events_Count`, now - 600e3, now).catch(() => []);
                return pts.reduce((a, p) => a + (+p.val || 0), 0);
            })
        );
        mount(
            el,
            h(
                'div',
                { class: 'dash-row' },
                h('div', { class: 'widget' }, h('div', { class: 'title' }, 'Flows'), h('div', { class: 'big' }, String((flows || []).length))),
                h('div', { class: 'widget' }, h('div', { class: 'title' }, 'Jobs running'), h('div', { class: 'big' }, `${running.length} / ${(jobs || []).length}`)),
                h('div', { class: 'widget' }, h('div', { class: 'title' }, 'Events, last 10 min'),
                    h('div', { class: 'big' }, formatters.longint(rates.reduce((a, b) => a + b, 0))))
            ),
            (flows || []).length
                ? h('ul', null, flows.map((f, i) => h('li', null, h('a', { href: `/config/edit/${f.name}`, 'data-nav': true }, f.displayName || f.name),
                    ' — ', formatters.longint(rates[i]), ' events in the last 10 min · ',
                    h('a', { href: `/dashboard/${f.name}`, 'data-nav': true }, 'metrics'))))
                : h('div', { class: 'muted' }, 'No flows yet.')
        );
    } catch (e) {
        mount(el, MessageBar('error', e.message));
    }
}
